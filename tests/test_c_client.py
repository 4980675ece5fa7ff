"""The C ABI driven from plain C (tests/c_client/fbm_c_roundtrip.c): the header compiles as strict C99,
the client links the in-tree library and agrees on the ABI (CPU), and -- on the GPU -- a C program that
allocates its own device buffers runs both crypters' round trip (every party's fbm_jl_encrypt /
fbm_lom_protect, then fbm_jl_aggregate / fbm_lom_aggregate) with results bit-identical to the oracle
(oracle/secagg_oracle.py, pinned by tests/golden/) and to the Python API on the same inputs.  This is the
boundary a non-Python host (cgo, JNI, N-API) would bind; INTEGRATION.md shows the ctypes one.  The client
also runs the Joye-Libert round with every factor computed ahead (fbm_jl_decrypt_factor ->
fbm_jl_encrypt_factor / fbm_jl_aggregate_factor, ABI 5) and exits non-zero unless its bytes are the same."""

import os
import random
import shutil
import struct
import subprocess

import numpy as np
import pytest

from fedbiomed_amd import _build, _device as D, workload as W
from fedbiomed_amd.constants import SAParameters

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fbm_secagg.h")


def _abi_version_in_header():
    for line in open(HEADER):
        if line.startswith("#define FBM_ABI_VERSION"):
            return int(line.split()[2])
    raise AssertionError("no FBM_ABI_VERSION in the header")


def test_header_is_strict_c99(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    src = tmp_path / "h.c"
    src.write_text('#include "fbm_secagg.h"\nint main(void) { return fbm_abi_version() == FBM_ABI_VERSION ? 0 : 1; }\n')
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                    "-I" + os.path.dirname(HEADER), str(src)], check=True)


def test_c_client_links_and_agrees_on_abi():
    """The built client resolves every entry point it calls from the in-tree library (the dynamic
    linker binds them at start-up) and reads the same ABI version as the header; no device touched."""
    if not os.path.exists(_build.CCLIENT_OUT):
        pytest.skip("C client not built (python -m fedbiomed_amd._build)")
    r = subprocess.run([_build.CCLIENT_OUT, "--abi"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert int(r.stdout) == _abi_version_in_header()


def _limbs(v, n):
    return int(v).to_bytes(4 * n, "little")


def _case(seed):
    rng = random.Random(seed)
    P = rng.randint(2, 5)
    n = (1, 7, 257, 3000)[seed % 4]
    target = rng.choice([None, 2**16, 2**20])
    clip = rng.choice([None, 1, 3])
    tr = target or SAParameters.TARGET_RANGE
    es, cr = D.jl_slot(tr, P)
    c, c2, tf, tm1 = D.quant_params(clip, tr)
    negc, step = D.dequant_params(clip, tr)
    weights = [rng.randint(1, 2**17 - 1) for _ in range(P)]
    keys = [rng.getrandbits(rng.choice([64, 2040])) for _ in range(P)]
    sk0 = -sum(keys)
    scale = (clip or SAParameters.CLIPPING_RANGE) * 1.2
    x = np.asarray([[rng.uniform(-scale, scale) for _ in range(n)] for _ in range(P)], np.float32)
    jl_tau, lom_tau = rng.getrandbits(40), rng.getrandbits(32)
    ids = W.node_ids(P)
    nonce = b"secagg_c_client"[:16].rjust(16, b"0")
    return dict(P=P, n=n, target=target, tr=tr, clip=clip, es=es, cr=cr, q=(c, c2, tf, tm1), dq=(negc, step),
                weights=weights, keys=keys, sk0=sk0, x=x, jl_tau=jl_tau, lom_tau=lom_tau, ids=ids, nonce=nonce)


def _write_case(path, k):
    P, n = k["P"], k["n"]
    c, c2, tf, tm1 = k["q"]
    negc, step = k["dq"]
    total = sum(k["weights"])
    with open(path, "wb") as f:
        f.write(b"FBMCRT1\0")
        f.write(struct.pack("<4I", P, k["es"], k["cr"], 0))
        f.write(struct.pack("<5Q", n, n, tm1, total, k["lom_tau"]))
        f.write(struct.pack("<5d", c, c2, tf, negc, step))
        f.write(_limbs(W.BIPRIME0, 32) + _limbs(k["jl_tau"], 256) + _limbs(abs(k["sk0"]), 64))
        f.write(struct.pack("<2i", 1 if k["sk0"] < 0 else 0, 0))
        for p in range(P):
            f.write(struct.pack("<Q2i", k["weights"][p], 0, 0) + _limbs(k["keys"][p], 64))
        f.write(k["x"].tobytes())
        f.write(k["nonce"])
        for p, u in enumerate(k["ids"]):
            sec = W.pairwise_secrets_for(u, k["ids"])
            peers = [o for o in k["ids"] if o != u]
            f.write(b"".join(sec[o] for o in peers))
            f.write(np.asarray([1 if o < u else -1 for o in peers], np.int8).tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_c_client_round_trip_vs_oracle(seed, tmp_path):
    from oracle import secagg_oracle as O

    assert os.path.exists(_build.CCLIENT_OUT), "C client not built (python -m fedbiomed_amd._build)"
    k = _case(4400 + seed)
    P, n, cr = k["P"], k["n"], k["cr"]
    n_ct = -(-n // cr)
    inp, outp = tmp_path / "case.bin", tmp_path / "out.bin"
    _write_case(inp, k)
    r = subprocess.run([_build.CCLIENT_OUT, str(inp), str(outp)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    blob = outp.read_bytes()
    sizes = [P * n_ct * 256, 8 * n, 8 * P * n, 8 * n]
    assert len(blob) == sum(sizes)
    o = np.cumsum([0] + sizes)
    cts = np.frombuffer(blob[o[0]:o[1]], np.uint32).reshape(P, n_ct, 64)
    jl_avg = np.frombuffer(blob[o[1]:o[2]], np.float64)
    lom_y = np.frombuffer(blob[o[2]:o[3]], np.uint64).reshape(P, n)
    lom_avg = np.frombuffer(blob[o[3]:o[4]], np.float64)
    total = sum(k["weights"])
    xs = [k["x"][p].astype(np.float64) for p in range(P)]

    ref_cts = [O.jl_encrypt(xs[p].tolist(), k["jl_tau"], k["keys"][p], W.BIPRIME0, P, clip=k["clip"],
                            weight=k["weights"][p], target=k["target"]) for p in range(P)]
    for p in range(P):
        assert D.limbs_to_ints(np.ascontiguousarray(cts[p])) == ref_cts[p], (seed, p)
    ref_avg = O.jl_crypter_aggregate(ref_cts, k["jl_tau"], k["sk0"], W.BIPRIME0, total, n, clip=k["clip"],
                                     target=k["target"])
    assert jl_avg.view(np.uint64).tolist() == np.asarray(ref_avg, np.float64).view(np.uint64).tolist(), seed

    ys = []
    for p, u in enumerate(k["ids"]):
        ref_y = np.asarray(O.lom_encrypt(xs[p], k["lom_tau"], u, W.pairwise_secrets_for(u, k["ids"]), k["ids"],
                                         k["nonce"], clip=k["clip"], weight=k["weights"][p], target=k["target"]),
                           np.uint64)
        assert lom_y[p].tolist() == ref_y.tolist(), (seed, p)
        ys.append(ref_y)
    ref_lom = O.lom_crypter_aggregate(ys, total, clip=k["clip"], target=k["target"])
    assert lom_avg.view(np.uint64).tolist() == np.asarray(ref_lom, np.float64).view(np.uint64).tolist(), seed

    # and the Python API on the same inputs: the same bytes through ctypes
    from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter

    jc = SecaggCrypter()
    got = [jc.encrypt(P, k["jl_tau"], xs[p].tolist(), k["keys"][p], W.BIPRIME0, clipping_range=k["clip"],
                      weight=k["weights"][p], target_range=k["target"]) for p in range(P)]
    assert got == ref_cts, seed
    lc = SecaggLomCrypter(k["nonce"].decode())
    assert O.lom_nonce(k["nonce"].decode()) == k["nonce"]
    for p, u in enumerate(k["ids"]):
        y = lc.encrypt(k["lom_tau"], u, xs[p].tolist(), W.pairwise_secrets_for(u, k["ids"]), k["ids"],
                       clipping_range=k["clip"], weight=k["weights"][p], target_range=k["target"])
        assert y == lom_y[p].tolist(), (seed, p)
