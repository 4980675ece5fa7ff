"""Batched exponentiation (fbm_jl_batch_begin / _flush, D.jl_exp_batch): several parties'
encrypt exponentiations and the decryption factor recorded inside the context run as ONE
jl_exp_kernel launch over all their chunks.  Results must be bit-identical to the per-call
launches (and to the oracle); calls the batch cannot take (a negative-key encrypt, whole
encrypts) launch as usual inside it; misuse is refused, not miscomputed."""

import pytest
import torch

from fedbiomed_amd import _device as D, _native, workload as W
from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError
from oracle import secagg_oracle as O


def test_batch_api_host():
    """No GPU: begin / abort bookkeeping and the workspace size."""
    from fedbiomed_amd import _build

    _build.build()
    lib = _native.load()
    assert lib.fbm_jl_batch_begin() == _native.FBM_OK
    assert lib.fbm_jl_batch_begin() == _native.FBM_E_ARG  # one open batch per thread
    lib.fbm_jl_batch_abort()
    assert lib.fbm_jl_batch_flush(None, 0, None) == _native.FBM_E_ARG  # nothing open
    assert lib.fbm_jl_batch_workspace() > 4096


def _pend_all(jc, xs, keys, ws, P, tau, off=0):
    return [jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p], ct_offset=off, defer_exp=True)
            for p in range(len(xs))]


@pytest.mark.gpu
def test_batch_equals_per_call():
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau = 4, 3
    sizes = [3_001, 77, 40_000, 257]  # different chunk counts per segment (incl. partial chunks)
    keys = [W.jl_user_key(p) for p in range(P)]
    keys[3] = 0  # a zero key takes the key_is_zero path inside the batch
    ws = [W.party_weight(p) for p in range(P)]
    xs = [torch.from_numpy(W.party_params(p, sizes[p])).to(dev) for p in range(P)]
    jc = SecaggCrypter()
    sk0 = -sum(keys)
    with D.jl_engine("single"):
        ref = [jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
        fref = jc.decrypt_factor_tensor(tau, 1_500, sk0, W.BIPRIME0, ct_offset=9)
    with D.deferred_checks():
        pend = _pend_all(jc, xs, keys, ws, P, tau)
        pf = jc.decrypt_factor_tensor(tau, 1_500, sk0, W.BIPRIME0, ct_offset=9, phased=True)
        with D.jl_exp_batch(dev):
            cts = [pend[p].finish() for p in range(P)]
            pf.exponentiate()
        f = pf.finish()  # sk0 < 0: the inverse, after the batch's launch
    for p in range(P):
        assert torch.equal(cts[p], ref[p]), p
    assert torch.equal(f, fref)
    es, cr = O.jl_slot(None, P)
    for p in (0, 2):  # first / last ciphertext of two parties vs the oracle
        qw = [int(v) * ws[p] for v in O.quantize(W.party_params(p, sizes[p]).astype("float64"))]
        for k in (0, cts[p].shape[0] - 1):
            got = D.limbs_to_ints(cts[p][k:k + 1].cpu().numpy())[0]
            assert got == O.jl_encrypt_ints(qw[k * cr:(k + 1) * cr], tau, keys[p], W.BIPRIME0, P, k0=k)[0]
    n2 = W.BIPRIME0 ** 2
    got = D.limbs_to_ints(f[[0, 1_499]].cpu().numpy())
    for g, k in zip(got, (9, 9 + 1_499)):
        assert g == O.powmod(O.fdh((k << 512) | tau, n2), sk0, n2)


@pytest.mark.gpu
def test_batch_mixed_and_refused_calls():
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau, n = 3, 1, 2_000
    keys = [W.jl_user_key(p) for p in range(P)]
    keys[1] = -keys[1]  # a negative-key encrypt is not deferred into the batch: it launches inline
    ws = [W.party_weight(p) for p in range(P)]
    xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
    jc = SecaggCrypter()
    ref = [jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
    with D.deferred_checks():
        pend = _pend_all(jc, xs, keys, ws, P, tau)
        with D.jl_exp_batch(dev):
            cts = [pend[p].finish() for p in range(P)]
            whole = jc.encrypt_tensor(P, tau, xs[0], keys[0], W.BIPRIME0, weight=ws[0])  # launches as usual
    for p in range(P):
        assert torch.equal(cts[p], ref[p]), p
    assert torch.equal(whole, ref[0])
    # a factor's inverse inside the open batch is refused (its exponentiation has not run yet)
    pf = jc.decrypt_factor_tensor(tau, 100, -123456789, W.BIPRIME0, phased=True)
    with pytest.raises(FedbiomedSecaggCrypterError):
        with D.jl_exp_batch(dev):
            pf.exponentiate()
            pf.finish()
    # a second biprime in one batch is refused
    other = W.BIPRIME0 - 2
    p1 = jc.encrypt_tensor(P, tau, xs[0], keys[0], W.BIPRIME0, weight=ws[0], defer_exp=True)
    p2 = jc.encrypt_tensor(P, tau, xs[2], keys[2], other, weight=ws[2], defer_exp=True)
    with pytest.raises(FedbiomedSecaggCrypterError):
        with D.jl_exp_batch(dev):
            p1.finish()
            p2.finish()
    torch.cuda.synchronize()
