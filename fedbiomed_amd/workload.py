"""Synthetic secagg workloads (SURVEY.md §8(d) "Synthetic inputs").

Shared by `bench.py`, the parity tests and `tools/gen_golden.py` so that every leg
(reference, oracle, HIP path) sees byte-identical inputs.  Pure numpy / stdlib.

* party p parameters: ``default_rng(1000+p).standard_normal(N).astype(float32) * 0.05``,
  then 0.1 % of the entries (index set drawn from the same rng) set to +/-4.0 so the
  clipping branch of ``quantize`` is exercised (c = 3);
* weights ``w_p = 1000 + 37 p``;
* LOM: node ids ``node-00 .. node-NN``; pairwise secret of (a, b) =
  ``SHA256(f"{min(a,b)}:{max(a,b)}")``; nonce string ``"secagg_0f1e2d3c4b5a"``;
* JL: default biprime0 (1024-bit, `envs/common/default_biprimes/biprime0.json` of the
  reference, a public parameter copied as a number below); user keys
  ``random.Random(7000+p).getrandbits(2040)``; server key ``-sum(user keys)``.
"""

import hashlib
import random
from typing import Dict, List

import numpy as np

# Public JL modulus shipped by the reference (envs/common/default_biprimes/biprime0.json;
# also `tests/test_secagg_crypter.py:14`).  1024 bits.
BIPRIME0 = int(
    "15882090880927171667165988061336610467781334125548783415430390976110721528356999552381742840298796264142"
    "9395032343305343341950966867458277812575065022203120547706127493272939455658018882112230042773163870472"
    "621818892994896895819790062496734944602899772583591514631486212290112369502692304700112819186167541107"
)

LOM_NONCE = "secagg_0f1e2d3c4b5a"


def party_params(p: int, n: int) -> np.ndarray:
    rng = np.random.default_rng(1000 + p)
    x = rng.standard_normal(n).astype(np.float32) * np.float32(0.05)
    k = max(1, n // 1000) if n >= 1000 else 0
    if k:
        idx = rng.choice(n, size=k, replace=False)
        sgn = rng.integers(0, 2, size=k)
        x[idx] = np.where(sgn == 1, np.float32(4.0), np.float32(-4.0))
    return x


def party_weight(p: int) -> int:
    return 1000 + 37 * p


def node_ids(n_parties: int) -> List[str]:
    return [f"node-{i:02d}" for i in range(n_parties)]


def pairwise_secret(a: str, b: str) -> bytes:
    lo, hi = (a, b) if a < b else (b, a)
    return hashlib.sha256(f"{lo}:{hi}".encode()).digest()


def pairwise_secrets_for(node: str, ids: List[str]) -> Dict[str, bytes]:
    return {o: pairwise_secret(node, o) for o in ids if o != node}


def jl_user_key(p: int) -> int:
    return random.Random(7000 + p).getrandbits(2040)


def jl_server_key(n_parties: int) -> int:
    return -sum(jl_user_key(p) for p in range(n_parties))
