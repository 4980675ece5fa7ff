"""The C ABI's argument checks from a caller that gets things wrong (include/fbm_secagg.h: "return value:
FBM_OK or a negative FBM_E_* code; fbm_last_error() has the message"): null pointers, bad dtypes, bad VES
parameters, out-of-range weights, node counts and phases, moduli an entry point does not take, ciphertext
counts past FBM_JL_MAX_CT -- each refused with its code and a message before any kernel runs, and the
library still computing correctly afterwards (no sticky state).  Device buffers are valid throughout (only
the argument under test is wrong), so nothing here can fault the GPU."""
import ctypes

import numpy as np
import pytest
import torch

from fedbiomed_amd import _device as D, _native as N, workload as W

E_ARG, E_UNSUPPORTED = -1, -8


@pytest.fixture(scope="module")
def env():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lib = N.load()
    dev = D.device()
    n_ct = 4
    st = torch.zeros(4, dtype=torch.int32, device=dev)
    ws = torch.empty(int(max(lib.fbm_jl_encrypt_workspace(n_ct), lib.fbm_jl_aggregate_workspace(n_ct))),
                     dtype=torch.uint8, device=dev)
    x = torch.zeros(n_ct, dtype=torch.float32, device=dev)
    ct = torch.empty((2, n_ct, 64), dtype=torch.int32, device=dev)
    f = torch.empty((n_ct, 64), dtype=torch.int32, device=dev)
    out = torch.empty(n_ct, dtype=torch.float64, device=dev)
    host = {"bp": D.int_limbs(W.BIPRIME0, 32), "even": D.int_limbs(W.BIPRIME0 + 1, 32),
            "key": D.int_limbs(W.jl_user_key(0), 64), "tau": D.int_limbs(3, N.TAU_LIMBS),
            "sec": np.zeros(32, np.uint8), "nonce": np.zeros(16, np.uint8), "signs": np.ones(1, np.int8)}
    return lib, dev, n_ct, st, ws, x, ct, f, out, host


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _h(a):
    return ctypes.c_void_p(a.ctypes.data)


def _q():  # clip 3, target 2^13: float(c), float(2c), float(T), T - 1
    return 3.0, 6.0, 8192.0, 8191


def _expect(lib, rc, code):
    assert rc == code, (rc, code, lib.fbm_last_error())
    assert lib.fbm_last_error(), "no message"


def _encrypt(lib, x, n, dtype, es, cr, weight, bp, key, tau, ct, ws, st, s=None):
    c, c2, tf, tm1 = _q()
    return lib.fbm_jl_encrypt(x, dtype, n, c, c2, tf, tm1, weight & (2**64 - 1), es, cr, bp, key, 0, tau, 0, ct, ws,
                              st, s)


@pytest.mark.gpu
def test_jl_encrypt_refusals(env):
    lib, dev, n_ct, st, ws, x, ct, f, out, h = env
    es, cr = D.jl_slot(None, 2)
    bp, key, tau = _h(h["bp"]), _h(h["key"]), _h(h["tau"])
    args = dict(x=_p(x), n=n_ct, dtype=N.FBM_F32, es=es, cr=cr, weight=1, bp=bp, key=key, tau=tau, ct=_p(ct[0]),
                ws=_p(ws), st=_p(st))
    for change, code in (({"x": None}, E_ARG), ({"dtype": 99}, E_ARG), ({"tau": None}, E_ARG),
                         ({"bp": None}, E_ARG), ({"key": None}, E_ARG), ({"cr": 0}, E_ARG),
                         ({"ws": None}, E_ARG), ({"ct": None}, E_ARG), ({"weight": -(2**17)}, E_ARG),
                         ({"es": 0}, E_ARG), ({"es": 101}, E_ARG),
                         ({"n": 14_000_001, "cr": 1, "es": 30}, E_UNSUPPORTED)):  # past FBM_JL_MAX_CT
        _expect(lib, _encrypt(lib, **{**args, **change}), code)
    c, c2, tf, tm1 = _q()
    _expect(lib, lib.fbm_jl_encrypt_phase(_p(x), N.FBM_F32, n_ct, c, c2, tf, tm1, 1, es, cr, bp, key, 0, tau, 0,
                                          _p(ct[0]), _p(ws), _p(st), None, 4), E_ARG)  # phases are 1, 2, 3
    # and the library still encrypts: the same as the Python layer's call
    assert _encrypt(lib, **args) == 0
    torch.cuda.synchronize()
    ref = D.jl_encrypt(x, W.BIPRIME0, W.jl_user_key(0), 3, 2, clip=3, target=8192)
    assert torch.equal(ct[0][:ref.shape[0]], ref)


@pytest.mark.gpu
def test_factor_and_aggregate_refusals(env):
    lib, dev, n_ct, st, ws, x, ct, f, out, h = env
    es, cr = D.jl_slot(None, 2)
    bp, key, tau = _h(h["bp"]), _h(h["key"]), _h(h["tau"])
    c, c2, tf, tm1 = _q()
    enc_f = dict(x=_p(x), n=n_ct, bp=bp, f=_p(f), ct=_p(ct[0]), ws=_p(ws))
    for change, code in (({"bp": _h(h["even"])}, E_UNSUPPORTED), ({"f": None}, E_ARG), ({"x": None}, E_ARG),
                         ({"ws": None}, E_ARG), ({"ct": _p(f)}, E_ARG)):  # (the output staged over the factor)
        a = {**enc_f, **change}
        _expect(lib, lib.fbm_jl_encrypt_factor(a["x"], N.FBM_F32, a["n"], c, c2, tf, tm1, 1, es, cr, a["bp"], a["f"],
                                               a["ct"], a["ws"], _p(st), None), code)
    _expect(lib, lib.fbm_jl_decrypt_factor(n_ct, bp, None, 0, tau, 0, _p(f), _p(ws), _p(st), None), E_ARG)
    _expect(lib, lib.fbm_jl_decrypt_factor(n_ct, None, key, 0, tau, 0, _p(f), _p(ws), _p(st), None), E_ARG)
    for phase in (0, 8):
        _expect(lib, lib.fbm_jl_decrypt_factor_phase(n_ct, bp, key, 0, tau, 0, _p(f), _p(ws), _p(st), None, phase),
                E_ARG)
    negc, step = D.dequant_params(3, 8192)
    agg = dict(cts=_p(ct), P=2, bp=bp, key=key, tw=2, ws=_p(ws))
    for change in ({"P": 0}, {"tw": 0}, {"key": None}, {"cts": None}, {"bp": None}, {"ws": None}):
        a = {**agg, **change}
        _expect(lib, lib.fbm_jl_aggregate(a["cts"], a["P"], n_ct, es, cr, n_ct * cr, a["bp"], a["key"], 1, tau, 0,
                                          a["tw"], negc, step, _p(out), None, a["ws"], _p(st), None), E_ARG)
    _expect(lib, lib.fbm_jl_aggregate_factor(_p(ct), 2, n_ct, es, cr, n_ct * cr, bp, None, 2, negc, step, _p(out),
                                             None, _p(ws), _p(st), None), E_ARG)
    _expect(lib, lib.fbm_jl_product(_p(ct), 0, n_ct, bp, _p(f), _p(ws), None), E_ARG)


@pytest.mark.gpu
def test_lom_and_helpers_refusals(env):
    lib, dev, n_ct, st, ws, x, ct, f, out, h = env
    c, c2, tf, tm1 = _q()
    y = torch.empty((2, n_ct), dtype=torch.int64, device=dev)
    negc, step = D.dequant_params(3, 8192)
    _expect(lib, lib.fbm_lom_aggregate(_p(y), 0, n_ct, 2, negc, step, _p(out), None, _p(st), None), E_ARG)
    _expect(lib, lib.fbm_lom_aggregate(_p(y), 2, n_ct, 0, negc, step, _p(out), None, _p(st), None), E_ARG)
    _expect(lib, lib.fbm_lom_aggregate(None, 2, n_ct, 2, negc, step, _p(out), None, _p(st), None), E_ARG)
    _expect(lib, lib.fbm_prf_key(None, _h(h["nonce"]), 1, _p(f), None), E_ARG)
    _expect(lib, lib.fbm_prf_key(_h(h["sec"]), None, 1, _p(f), None), E_ARG)
    _expect(lib, lib.fbm_dequantize(None, n_ct, negc, step, _p(out), None), E_ARG)
    # and the LOM path still computes: the Python layer's protect + aggregate agree with the oracle elsewhere;
    # here the aggregate of zeros is the clipping floor's dequantised mean
    y.zero_()
    assert lib.fbm_lom_aggregate(_p(y), 2, n_ct, 2, negc, step, _p(out), None, _p(st), None) == 0
    torch.cuda.synchronize()
    assert out.cpu().tolist() == [negc] * n_ct
