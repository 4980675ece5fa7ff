"""GPU smoke of the batched exponentiation: two parties recorded in one launch vs per-call launches."""
import sys

import torch

sys.path.insert(0, '.')
from fedbiomed_amd import _device as D, workload as W  # noqa: E402
from fedbiomed_amd.secagg import SecaggCrypter  # noqa: E402

dev = D.device()
jc = SecaggCrypter()
x = torch.from_numpy(W.party_params(0, 1000)).to(dev)
with D.jl_engine("single"), D.deferred_checks():
    ref = [jc.encrypt_tensor(2, 1, x[:n], W.jl_user_key(p), W.BIPRIME0, weight=3) for p, n in ((0, 1000), (1, 300))]
    pend = [jc.encrypt_tensor(2, 1, x[:n], W.jl_user_key(p), W.BIPRIME0, weight=3, defer_exp=True)
            for p, n in ((0, 1000), (1, 300))]
    with D.jl_exp_batch(dev):
        got = [q.finish() for q in pend]
    torch.cuda.synchronize()
print("batch equal:", all(torch.equal(a, b) for a, b in zip(ref, got)), flush=True)
