"""The LOM object API (fedbiomed_amd.secagg.LOM / PRF / SecaggLomCrypter) through the reference's
own test flows (tests/test_lom.py), restated for the mirror, plus the same flows checked against
the oracle (bit-exact masked vectors).  Every call runs the HIP kernels."""

import functools
import math
import random

import numpy as np
import pytest

from fedbiomed_amd.constants import SAParameters
from fedbiomed_amd.exceptions import FedbiomedSecaggError
from fedbiomed_amd.secagg import LOM, PRF, SecaggLomCrypter

pytestmark = pytest.mark.gpu

NODE_IDS = ["node-1", "node-2", "node-3"]
PWKEYS = ({"node-2": b"\x02" * 32, "node-3": b"\x02" * 32},
          {"node-1": b"\x02" * 32, "node-3": b"\x02" * 32},
          {"node-1": b"\x02" * 32, "node-2": b"\x02" * 32})
NONCE = bytes(range(16))


def test_prf_sizes_and_oracle():
    """reference test_lom.py:32-52, and the keystream vs the oracle"""
    from oracle import secagg_oracle as O

    prf = PRF(b"\x00" * 16)
    key = prf.eval_key(b"\x01" * 32, 1)
    assert len(key) == 32 and key == O.prf_eval_key(b"\x01" * 32, b"\x00" * 16, 1)
    for size in (10, 10000):
        vec = np.frombuffer(prf.eval_vector(key, 1, size), dtype="uint64")
        assert len(vec) == size
        assert vec.tolist() == O.prf_eval_vector(key, b"\x00" * 16, 1, size).tolist()


def test_lom_protect_and_aggregate():
    """reference test_lom.py:55-78 (+ the masked vectors bit-exact vs the oracle)"""
    from oracle import secagg_oracle as O

    xs = ([11111, 21111, 311111, 41111, 51111, 11116], [23131231, 1231232, 2342343, 32434, 2432345, 2343246],
          [2343241, 2342342, 4443, 34444, 2225, 2342346])
    ys = [LOM(nonce=NONCE).protect(NODE_IDS[u], PWKEYS[u], 1, list(xs[u]), NODE_IDS) for u in range(3)]
    for u in range(3):
        assert len(ys[u]) == len(xs[u])
        assert ys[u] == [int(v) for v in O.lom_protect(NODE_IDS[u], PWKEYS[u], 1, xs[u], NODE_IDS, NONCE)]
    assert LOM(nonce=NONCE).aggregate(ys) == np.sum(np.array(xs), axis=0).tolist()
    LOM(NONCE).protect(NODE_IDS[0], PWKEYS[0], 1, [112341234, 123151234], NODE_IDS)  # test_lom.py:81-89


def test_lom_protect_big_int():
    """reference test_lom.py:92-126: 26-bit values round-trip, 62-bit values overflow (FB417)"""
    r = random.Random(3).getrandbits(26)
    params = [r, r]
    ys = [LOM(nonce=NONCE).protect(NODE_IDS[u], PWKEYS[u], 1, params, NODE_IDS) for u in range(3)]
    assert LOM(nonce=NONCE).aggregate(ys) == [3 * r, 3 * r]
    r62 = (1 << 61) | random.Random(4).getrandbits(61)
    with pytest.raises(FedbiomedSecaggError):
        LOM(nonce=NONCE).protect(NODE_IDS[0], PWKEYS[0], 1, [r62, r62], NODE_IDS)


def test_lom_crypter_round_trip():
    """reference test_lom.py:129-153"""
    cr = SecaggLomCrypter("a-url-safe-nonce-123")
    params = [1.5, 1.5, 1.5, 1.5, 1.5]
    enc = functools.partial(cr.encrypt, current_round=1, node_ids=NODE_IDS, params=params, weight=1)
    e = [enc(node_id=NODE_IDS[i], pairwise_secrets=PWKEYS[i]) for i in range(3)]
    result = cr.aggregate(e, 3)
    assert all(math.isclose(v1, v2, rel_tol=0.01) for v1, v2 in zip(result, params))


def test_lom_crypter_target_range_precision():
    """reference test_lom.py:156-187: FA_TARGET_RANGE recovers large values, the default is too coarse"""
    cr = SecaggLomCrypter("another-nonce")
    params = [123456.0, -98765.0, 4321.0]

    def round_trip(target_range):
        enc = functools.partial(cr.encrypt, current_round=1, node_ids=NODE_IDS, params=params, weight=1,
                                clipping_range=1_000_000, target_range=target_range)
        e = [enc(node_id=NODE_IDS[i], pairwise_secrets=PWKEYS[i]) for i in range(3)]
        return cr.aggregate(e, 3, clipping_range=1_000_000, target_range=target_range)

    fa = round_trip(SAParameters.FA_TARGET_RANGE)
    assert all(math.isclose(g, e, abs_tol=1.0) for g, e in zip(fa, params))
    default = round_trip(None)
    assert not all(math.isclose(g, e, abs_tol=1.0) for g, e in zip(default, params))
