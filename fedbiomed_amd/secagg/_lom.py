"""LOM / PRF objects mirroring the reference class API (fedbiomed/common/secagg/_lom.py),
for callers and tests that use them directly.  All keystream and mask arithmetic runs in
the gfx950 kernels (fbm_lom_protect / fbm_prf_key)."""

import math
import secrets
from typing import Dict, List

import numpy as np
import torch

from .. import _device as D
from ..constants import ErrorNumbers
from ..exceptions import FedbiomedSecaggError  # noqa: F401  (raised by D's helpers; the API's error class)

_MAX_ROUND = 1000


class PRF:
    def __init__(self, nonce: bytes) -> None:
        self._nonce = nonce

    def eval_key(self, pairwise_secret: bytes, tau: int) -> bytes:
        """reference _lom.py:30-56"""
        return D.prf_key(pairwise_secret, self._nonce, tau)

    def eval_vector(self, seed: bytes, tau: int, input_size: int) -> bytes:
        """reference _lom.py:58-83: keystream XOR (i+tau).to_bytes(8,'big'), as bytes."""
        if not (input_size + _MAX_ROUND) <= 2**61:
            raise FedbiomedSecaggError(
                f"{ErrorNumbers.FB417.value}: Can not perform encryiton due to large input vector. input_size "
                f"({input_size}) + MAX_ROUND ({_MAX_ROUND}) allowed is greater than 2**61 ")
        if input_size == 0:
            return b""
        dev = D.device()
        zeros = torch.zeros(input_size, dtype=torch.int64, device=dev)
        y = D.lom_protect(zeros, [seed], [1], self._nonce, tau, 1, weight=1, raw_seeds=True)
        return y.cpu().numpy().tobytes()


class LOM:
    def __init__(self, nonce: bytes = None) -> None:
        if not nonce:
            nonce = secrets.token_bytes(16)
        self._nonce = nonce
        self._prf = PRF(nonce)
        self._vector_dtype = "uint64"
        self._values_bit = 64

    def protect(self, node_id: str, pairwise_secrets: Dict[str, bytes], tau: int, x_u_tau: List[int],
                node_ids: List[str]) -> List[int]:
        """reference _lom.py:105-175 (integer input vector)."""
        num_nodes = len(node_ids)
        _max_param_bits = max(val.bit_length() for val in x_u_tau)
        _node_bits = math.ceil(math.log2(num_nodes))
        if _max_param_bits >= self._values_bit - _node_bits:  # the reference's message, word for word
            raise FedbiomedSecaggError(D._lom_overflow_message(_max_param_bits, num_nodes))
        x = D.u64_to_device(list(x_u_tau))
        peers = [p for p in node_ids if p != node_id]
        y = D.lom_protect(x, [pairwise_secrets[p] for p in peers], [1 if p < node_id else -1 for p in peers],
                          self._nonce, tau, num_nodes, weight=1)
        return D.u64_from_device(y)

    def aggregate(self, list_y_u_tau: List[List[int]]) -> List[int]:
        """reference _lom.py:177-192: u64 column sum mod 2^64."""
        Y = D.u64_to_device(list_y_u_tau)
        _, sums = D.lom_aggregate(Y, 1, want_out=False, want_sums=True)
        return sums.cpu().numpy().view(np.uint64).tolist()
