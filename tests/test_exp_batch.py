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


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [5, 300, 1000, 1024])
def test_batch_random_moduli(bits):
    """The batched launch on random odd moduli (small ones: FDH retries, i.e. wide digests
    entering as h_lo R + h_hi R^2 inside the batch), keys of several lengths incl. 0, and the
    decryption factor of a negative sum: bit-identical to per-call launches and the oracle."""
    import random

    dev = D.device()
    rng = random.Random(3000 + bits)
    N = max(3, rng.getrandbits(bits) | (1 << (bits - 1)) | 1)
    n2, P, tau = N * N, 3, rng.getrandbits(64)
    sizes = [37, 300, 1]
    keys = [rng.getrandbits(rng.choice([40, 700, 2040])) for _ in range(P)]
    keys[2] = 0
    xs = [torch.tensor([rng.getrandbits(63) for _ in range(s)], dtype=torch.int64, device=dev) for s in sizes]
    ref = [D.jl_encrypt(xs[p], N, keys[p], tau, P, slot=(100, 1)) for p in range(P)]
    sk0 = -sum(keys) - 1
    fref = D.jl_decrypt_factor(50, N, sk0, tau, ct_offset=4)
    with D.deferred_checks():
        pend = [D.jl_encrypt(xs[p], N, keys[p], tau, P, slot=(100, 1), defer_exp=True) for p in range(P)]
        pf = D.jl_decrypt_factor(50, N, sk0, tau, ct_offset=4, phased=True)
        with D.jl_exp_batch(dev):
            pf.exponentiate()
            cts = [q.finish() for q in pend]
        f = pf.finish()
    for p in range(P):
        assert torch.equal(cts[p], ref[p]), p
        k = sizes[p] - 1
        pt = int(xs[p][k])
        want = ((N * pt + 1) % n2) * O.powmod(O.fdh((k << 512) | tau, n2), keys[p], n2) % n2
        assert D.limbs_to_ints(cts[p][k:k + 1].cpu().numpy())[0] == want, p
    assert torch.equal(f, fref)
    got = D.limbs_to_ints(f[[0, 49]].cpu().numpy())
    for g, k in zip(got, (4, 53)):
        assert g == O.powmod(O.fdh((k << 512) | tau, n2), sk0, n2)


@pytest.mark.gpu
def test_batch_abort_invalidates_recorded_calls():
    """An exception inside jl_exp_batch drops the batch: the recorded exponentiations never run, so
    finish() on their Pending objects raises afterwards instead of handing out unwritten memory.
    Calls that launched at once inside the block (a negative-key encrypt, an even biprime on the
    generic engine) were not recorded and stay valid."""
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau, n = 3, 1, 1_000
    keys = [W.jl_user_key(p) for p in range(P)]
    keys[1] = -keys[1]
    ws = [W.party_weight(p) for p in range(P)]
    xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
    jc = SecaggCrypter()
    ref = [jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
    even = 1156
    ref_even = jc.encrypt_tensor(P, tau, xs[2], keys[2], even, weight=ws[2])
    pend = _pend_all(jc, xs, keys, ws, P, tau)
    pe = jc.encrypt_tensor(P, tau, xs[2], keys[2], even, weight=ws[2], defer_exp=True)
    pf = jc.decrypt_factor_tensor(tau, 100, -sum(keys), W.BIPRIME0, phased=True)
    with pytest.raises(KeyError):
        with D.jl_exp_batch(dev):
            out = [pend[p].finish() for p in range(P)]
            out_even = pe.finish()
            pf.exponentiate()
            raise KeyError("caller error inside the batch")
    for p in (0, 2):
        with pytest.raises(RuntimeError, match="aborted"):
            pend[p].finish()
    with pytest.raises(RuntimeError, match="aborted"):
        pf.finish()
    torch.cuda.synchronize()
    assert torch.equal(pend[1].finish(), ref[1]) and torch.equal(out[1], ref[1])  # negative key: ran inline
    assert torch.equal(pe.finish(), ref_even) and torch.equal(out_even, ref_even)  # generic engine: ran inline


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["single", "triple", "quad"])
def test_short_path_equals_table_path(engine):
    """The short path (binary chain, short-base products, the key's constant C: DESIGN.md 5.3) and the
    window-table path give the same ciphertexts and decryption factors bit for bit, under every engine:
    positive and negative keys, a key of one bit, the default biprime."""
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    n, P = 3000, 3
    xs = torch.from_numpy(W.party_params(7, n)).to(dev)
    jc = SecaggCrypter()
    out = {}
    for short in (True, False):
        with D.jl_short(short), D.jl_engine(engine):
            cts = [jc.encrypt_tensor(P, 5, xs, k, W.BIPRIME0, weight=3) for k in (W.jl_user_key(1), 1, 1 << 2039)]
            fac = [D.jl_decrypt_factor(700, W.BIPRIME0, k, 5, dev=dev) for k in (W.jl_server_key(P), -1, 2)]
            torch.cuda.synchronize()
            out[short] = [c.cpu() for c in cts] + [f.cpu() for f in fac]
    for a, b in zip(out[True], out[False]):
        assert torch.equal(a, b)


@pytest.fixture
def test_build():
    """The whole test through the test build (_native.test_hooks): a split call's phases must run in
    the library whose switches set its path, and whose records hold it."""
    from fedbiomed_amd import _native

    with _native.test_hooks():
        yield _native.load_test()


@pytest.mark.gpu
def test_split_calls_follow_their_phase1_path(test_build):
    """a split call (encrypt with defer_exp, a phased factor) takes the path its
    phase 1 set up -- generic or Montgomery engine, short path or table path -- even when the
    process-wide switches change before its later phases; and a batch whose first segment ran with the
    short path off still gives the short-path segments their D pairs.  Every result equals the
    unsplit call."""
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau, n = 3, 2, 1_500
    keys = [W.jl_user_key(p) for p in range(P)]
    ws = [W.party_weight(p) for p in range(P)]
    xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
    jc = SecaggCrypter()
    sk0 = -sum(keys)
    ref = [jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
    n_ct = ref[0].shape[0]
    fref = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0)
    switches = [lambda: D.jl_engine("generic"), lambda: D.jl_short(False)]
    for sw in switches:
        # the switch around phase 1 only
        with sw():
            pe = jc.encrypt_tensor(P, tau, xs[0], keys[0], W.BIPRIME0, weight=ws[0], defer_exp=True)
            pf = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0, phased=True)
        assert torch.equal(pe.finish(), ref[0])
        assert torch.equal(pf.exponentiate().finish(), fref)
        # the switch around the later phases only
        pe = jc.encrypt_tensor(P, tau, xs[1], keys[1], W.BIPRIME0, weight=ws[1], defer_exp=True)
        pf = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0, phased=True)
        with sw():
            c1 = pe.finish()
            pf.exponentiate()
            f = pf.finish()
        assert torch.equal(c1, ref[1]) and torch.equal(f, fref)
    # a batch: party 0's phase 1 with the short path off, the others' with it on
    with D.deferred_checks():
        with D.jl_short(False):
            pend = [jc.encrypt_tensor(P, tau, xs[0], keys[0], W.BIPRIME0, weight=ws[0], defer_exp=True)]
        pend += [jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p], defer_exp=True)
                 for p in range(1, P)]
        with D.jl_exp_batch(dev):
            cts = [q.finish() for q in pend]
    for p in range(P):
        assert torch.equal(cts[p], ref[p]), p
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_split_call_survives_clear_caches_and_refuses_unknown_workspace(test_build):
    """fbm_jl_clear_caches between a split call's phases leaves its phase-1 path
    record alone (the result equals the unsplit call's even with the switches changed in between),
    and a later phase on a workspace phase 1 never ran on is FBM_E_ARG, not a guess."""
    import ctypes

    from fedbiomed_amd import _native
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    lib = test_build
    P, tau, n = 2, 3, 900
    key = W.jl_user_key(0)
    x = torch.from_numpy(W.party_params(0, n)).to(dev)
    jc = SecaggCrypter()
    ref = jc.encrypt_tensor(P, tau, x, key, W.BIPRIME0)
    n_ct = ref.shape[0]
    sk0 = -key
    fref = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0)
    with D.jl_short(False):
        pe = jc.encrypt_tensor(P, tau, x, key, W.BIPRIME0, defer_exp=True)
        pf = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0, phased=True)
    lib.fbm_jl_clear_caches()
    assert torch.equal(pe.finish(), ref)
    assert torch.equal(pf.exponentiate().finish(), fref)
    # phase 2 of the factor on a fresh workspace: refused
    ws = torch.zeros(lib.fbm_jl_aggregate_workspace(n_ct), dtype=torch.uint8, device=dev)
    st = torch.zeros(_native.STATS_WORDS, dtype=torch.int32, device=dev)
    out = torch.empty((n_ct, 64), dtype=torch.int32, device=dev)
    nl = D.int_limbs(W.BIPRIME0, 32)
    kl = D.int_limbs(abs(sk0), 64)
    tl = D.int_limbs(tau, _native.TAU_LIMBS)
    rc = lib.fbm_jl_decrypt_factor_phase(n_ct, nl.ctypes.data, kl.ctypes.data, 1, tl.ctypes.data, 0,
                                         ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                         ctypes.c_void_p(st.data_ptr()),
                                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), 2)
    assert rc == _native.FBM_E_ARG
    assert "phase-1 record" in _native.last_error()
    torch.cuda.synchronize()
