"""The library keeps no key material between calls: the short
path's per-(N, |key|) constant C is cached under a SHA-256 digest of (N, |key|), the entry holds only
the digest and C, entries are zeroed on eviction, and fbm_jl_clear_caches() empties the cache.  The
reference keeps nothing (a fresh SecaggCrypter per call: fedbiomed/node/secagg/_secagg_round.py:142).
Host-only (no GPU): the cache is filled through the fbm_test_short_consts hook, which runs the same
build_short the JL entry points call."""

import hashlib
import random

import numpy as np

from fedbiomed_amd import _build, _native, workload as W

ENTRY_WORDS = 8 + 72


def _lib():
    _build.build()
    return _native.load_test()  # fbm_test_short_* (include/fbm_secagg_test.h)


def _consts(lib, N, key):
    n32 = np.frombuffer(N.to_bytes(128, "little"), dtype=np.uint32).copy()
    k64 = np.frombuffer(abs(key).to_bytes(256, "little"), dtype=np.uint32).copy()
    kw, corr, d = np.zeros(64, np.uint32), np.zeros(72, np.uint32), np.zeros(36, np.uint32)
    r = lib.fbm_test_short_consts(n32.ctypes.data, k64.ctypes.data, kw.ctypes.data, corr.ctypes.data, d.ctypes.data)
    assert r >= 0
    return corr


def _dump(lib):
    n = lib.fbm_test_short_cache(None, 0)
    assert n >= 0 and n % ENTRY_WORDS == 0
    out = np.zeros(max(n, 1), np.uint32)
    assert lib.fbm_test_short_cache(out.ctypes.data, n) == n
    return out[:n].reshape(-1, ENTRY_WORDS)


def test_cache_holds_digest_and_constant_only():
    lib = _lib()
    lib.fbm_jl_clear_caches()
    assert lib.fbm_test_short_cache(None, 0) == 0
    keys = [W.jl_user_key(p) for p in range(3)] + [W.jl_server_key(3)]
    corrs = [_consts(lib, W.BIPRIME0, k) for k in keys]
    ents = _dump(lib)
    assert ents.shape[0] == len(keys)
    blob = ents.tobytes()
    for k, corr, e in zip(keys, corrs, ents):
        kb = abs(k).to_bytes(256, "little")
        # no 16-byte window of the key's bytes appears anywhere in the cache
        assert not any(kb[i:i + 16] in blob for i in range(0, 256 - 16, 4) if any(kb[i:i + 16]))
        dg = hashlib.sha256(W.BIPRIME0.to_bytes(128, "little") + kb).digest()
        assert bytes(e[:8].astype(">u4").tobytes()) == dg  # SHA-256 state words, big-endian digest
        assert np.array_equal(e[8:], corr)
    # a repeated (N, key) is served from the cache (no new entry), with the same C
    assert np.array_equal(_consts(lib, W.BIPRIME0, keys[0]), corrs[0])
    assert _dump(lib).shape[0] == len(keys)
    lib.fbm_jl_clear_caches()
    assert lib.fbm_test_short_cache(None, 0) == 0
    # rebuilt after a clear: the same constant
    assert np.array_equal(_consts(lib, W.BIPRIME0, keys[1]), corrs[1])
    lib.fbm_jl_clear_caches()


def test_cache_is_bounded():
    lib = _lib()
    lib.fbm_jl_clear_caches()
    rng = random.Random(5)
    N = W.BIPRIME0
    for _ in range(34):
        _consts(lib, N, rng.getrandbits(300) | 1)
    assert _dump(lib).shape[0] == 32  # the oldest entries were evicted
    lib.fbm_jl_clear_caches()
    assert lib.fbm_test_short_cache(None, 0) == 0
