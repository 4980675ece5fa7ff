#!/usr/bin/env python3
"""Driver and checker of tools/microbench/mfma_redc.hip (round-5 VERDICT item 3: price the int8-MFMA
Montgomery reduction with a standalone kernel before any engine code).

Builds the inputs (T = t0 + H 2^1044 per ciphertext, t0 < 2^1044, H < 2^1021; the benchmark biprime N), the
constants (N's 29-bit limbs, the A fragments of the Toeplitz blocks of N' = -N^-1 mod R and of N in the MFMA
lane order, 7-bit digits, R = 2^1043), runs the kernel binary, replays its chain with Python integers --
m_bal = the balanced (digits in [-64, 63]) representative of T N' mod R, t = (T + (m_bal + R) N) / R, then
T <- t + H 2^1044 -- and checks every limb of a sample of ciphertexts bit for bit.  Prints one JSON line.

    python tools/microbench/mfma_redc_check.py [--ct 131072] [--iters 64] [--reps 5] [--check 512]
"""

import argparse
import json
import os
import random
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

ND, NL, R_BITS = 149, 36, 1043
R = 1 << R_BITS


def digits7(x, count):
    return [(x >> (7 * i)) & 127 for i in range(count)]


def a_fragments(digs, nd_valid, offsets):
    """[d][lane][16 bytes] A fragments: A[row][k] = digs[32 d + row - k] for 0 <= idx < nd_valid; lane l holds
    row l & 31, k = 16 (l >> 5) + j (the kernel's B operand uses the same k order)."""
    out = np.zeros((len(offsets), 64, 16), dtype=np.int8)
    for di, d in enumerate(offsets):
        for lane in range(64):
            row, h = lane & 31, lane >> 5
            for j in range(16):
                idx = 32 * d + row - (16 * h + j)
                if 0 <= idx < nd_valid:
                    out[di, lane, j] = digs[idx]
    return out


def limbs29(x, n):
    return [(x >> (29 * i)) & ((1 << 29) - 1) for i in range(n)]


def replay(T_low, H, N, Np, iters):
    off = 64 * (R - 1) // 127  # balanced digits in [-64, 63]: m_bal = ((T N' + off) mod R) - off
    t = T_low
    for _ in range(iters):
        T = t + (H << 1044)
        m = ((T * Np + off) % R) - off
        t = (T + (m + R) * N) // R
        assert (T + (m + R) * N) % R == 0
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ct", type=int, default=131072)
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=512)
    ap.add_argument("--bin", default=os.path.join(HERE, "mfma_redc"))
    args = ap.parse_args()
    from fedbiomed_amd import workload as W

    N = W.BIPRIME0
    Np = (-pow(N, -1, R)) % R
    n = args.ct
    rng = random.Random(5)
    T_low = [rng.getrandbits(1044) for _ in range(n)]
    H = [rng.getrandbits(1021) for _ in range(n)]
    Tarr = np.array([limbs29(x, NL) for x in T_low], dtype=np.uint32).T.copy()  # [36][n]
    Harr = np.array([limbs29(x, NL) for x in H], dtype=np.uint32).T.copy()
    Anp = a_fragments(digits7(Np, ND), ND, range(5))
    An = a_fragments(digits7(N, 147), 147, range(6))
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as fh:
            fh.write(struct.pack("<I", n))
            fh.write(Tarr.tobytes())
            fh.write(Harr.tobytes())
            fh.write(np.array(limbs29(N, NL), dtype=np.uint32).tobytes())
            fh.write(Anp.tobytes())
            fh.write(An.tobytes())
        r = subprocess.run([args.bin, fin, fout, str(args.iters), str(args.reps)], capture_output=True, text=True,
                           timeout=300)
        if r.returncode:
            print(r.stdout, r.stderr)
            sys.exit(1)
        lines = [json.loads(x) for x in r.stdout.strip().splitlines()]
        O = np.fromfile(fout, dtype=np.uint32).reshape(NL + 1, n)
    bad, sample = 0, rng.sample(range(n), min(args.check, n))
    for c in sample:
        want = replay(T_low[c], H[c], N, Np, args.iters)
        got = sum(int(O[L, c]) << (29 * L) for L in range(NL + 1))
        bad += got != want
    res = {"probe": lines[0], "timing": lines[1], "checked": len(sample), "mismatches": bad, "bit_exact": bad == 0}
    print(json.dumps(res))
    sys.exit(0 if bad == 0 else 2)


if __name__ == "__main__":
    main()
