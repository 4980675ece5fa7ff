"""Debug: batched vs per-party exponentiation at config-4 sizes (8 parties x 10M, +- the factor)."""
import sys

import torch

sys.path.insert(0, '.')
from fedbiomed_amd import _device as D, workload as W  # noqa: E402
from fedbiomed_amd.secagg import SecaggCrypter  # noqa: E402

dev = D.device()
jc = SecaggCrypter()
P, tau = 8, 1
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
keys = [W.jl_user_key(p) for p in range(P)]
ws = [W.party_weight(p) for p in range(P)]
sk0 = -sum(keys)
xd = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
ref = [jc.encrypt_tensor(P, tau, xd[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
n_ct = ref[0].shape[0]
fref = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0)
torch.cuda.synchronize()


def report(tag, got, fac):
    torch.cuda.synchronize()
    for p in range(P):
        bad = (got[p] != ref[p]).any(dim=1).nonzero().flatten()
        if bad.numel():
            print(f"{tag} p={p} n_ct={n_ct} bad={bad.numel()} first={bad[:6].tolist()} last={bad[-3:].tolist()}",
                  flush=True)
    if fac is not None:
        bad = (fac != fref).any(dim=1).nonzero().flatten()
        print(f"{tag} factor bad={bad.numel()} first={bad[:6].tolist()}", flush=True)
    print(f"{tag} done", flush=True)


for order in ("parties", "factor_first", "factor_last"):
    with D.deferred_checks():
        pend = [jc.encrypt_tensor(P, tau, xd[p], keys[p], W.BIPRIME0, weight=ws[p], defer_exp=True)
                for p in range(P)]
        pf = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0, phased=True) if order != "parties" else None
        with D.jl_exp_batch(dev):
            if order == "factor_first":
                pf.exponentiate()
            got = [q.finish() for q in pend]
            if order == "factor_last":
                pf.exponentiate()
        fac = pf.finish() if pf is not None else None
    report(order, got, fac)
    del pend, pf, got, fac
