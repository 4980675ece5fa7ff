"""Additive secret sharing of vectors on the MI355X (drop-in for the reference's
`fedbiomed/common/secagg/_additive_ss.py`).

`AdditiveSecret.split` (:40-98), `AdditiveShare.__add__` (:134-160) and
`AdditiveShares.reconstruct` (:252-267) keep the reference's classes, signatures, validation
and exceptions; the per-element work (share draws, exact sums) runs on the device:
`fbm_ass_split` / `fbm_ass_reconstruct` (int128 lanes) for secrets in [-2^63, 2^64) -- the
per-element vector use -- and `fbm_ass_split_wide` / `fbm_ass_reconstruct_wide`
(two's-complement u32 limbs of any width) for everything else, e.g. the 2040-bit JL user key
the key setup splits (`node/secagg/_secagg_setups.py:248-268`) and the server-key shares the
researcher sums (`researcher/secagg/_secagg_context.py:380-382`).

The reference draws shares from Python's MT19937 (`random.randint`, `_additive_ss.py:96`), a predictable
generator: its output reveals its state.  Here every secret -- an int (the JL key setup's only use,
`node/secagg/_secagg_setups.py:248-249`: a node's 2040-bit key) or a vector -- draws its shares from a
counter-based ChaCha20 stream on the device keyed from the OS (`os.urandom`), so a key's shares are not
predictable PRNG output (100M x 16 shares in milliseconds; MT19937 is sequential).  `reference_rng=True`
(an extension, for parity runs) draws them from the reference's own stream instead -- the global `random`'s
MT19937, call for call, so a seeded run gives the reference's shares exactly and leaves `random` in the
reference's state; the last share (secret - sum) is still computed on the device.  What both guarantee --
and what the tests pin -- is the contract: the shares sum exactly to the secret, the first n-1 lie in
[0, 2**bit_length].

`split_tensor` / `reconstruct_tensor` are the device fast path (int64 tensors in HBM).
"""

from __future__ import annotations

import random
from math import log2
from typing import List, Optional, Union

import numpy as np
import torch

from .. import _device as D
from ..exceptions import FedbiomedTypeError, FedbiomedValueError


def _in_64bit_domain(values: List[int]) -> bool:
    lo, hi = min(values), max(values)
    return not (lo < D.I64_MIN or hi >= D.U64_LIM or (lo < 0 and hi >= 2**63))


def _device_domain(values: List[int]) -> bool:
    """True -> uint64 input, False -> int64 input; raises outside [-2^63, 2^64)."""
    lo, hi = min(values), max(values)
    if lo < D.I64_MIN or hi >= D.U64_LIM or (lo < 0 and hi >= 2**63):
        raise FedbiomedValueError("The device additive secret sharing supports secrets in [-2^63, 2^63) "
                                  "or [0, 2^64)")
    return hi >= 2**63


class AdditiveSecret:
    """Manages additive secret (reference `_additive_ss.py:11-98`)."""

    def __init__(self, secret: Union[int, List[int]]) -> None:
        if not (isinstance(secret, int) or (isinstance(secret, list) and all(isinstance(i, int) for i in secret))):
            raise FedbiomedValueError("AdditiveSecret must be an int or a list of int")
        self._secret = secret

    @property
    def secret(self) -> Union[List, int]:
        return self._secret

    def split(self, num_shares: int, bit_length: Optional[int] = None,
              reference_rng: bool = False) -> "AdditiveShares":
        """`reference_rng` (an extension, for parity runs): the shares drawn from the reference's own
        stream (the global `random`'s MT19937: `random.randint` for an int secret, element by element
        through D.reference_share_draws for a vector) instead of the device's OS-keyed ChaCha20 --
        seeded, the reference's shares exactly; the last share is still computed on the device.  Off
        (the default), no share comes from `random`: a node's key shares are not predictable."""
        if num_shares <= 0:
            raise FedbiomedValueError("Number of shares must be greater than 0")
        values = [self._secret] if isinstance(self._secret, int) else list(self._secret)
        if bit_length is not None:
            for v in values:  # reference _shares_int check (log2 raises ValueError for v <= 0)
                if bit_length < int(log2(v)):
                    raise FedbiomedValueError("Bit length must be greater or equal than the secret's bit length")
        if not values:
            return AdditiveShares([AdditiveShare([]) for _ in range(num_shares)])
        if isinstance(self._secret, int) and reference_rng:  # the reference's own draws (:94-98), then secret - sum
            bl = self._secret.bit_length() if bit_length is None else bit_length
            draws = [random.randint(0, 2**bl) for _ in range(num_shares - 1)]
            last = _reconstruct([[self._secret]] + [[-d] for d in draws])[0]
            return AdditiveShares([AdditiveShare(d) for d in draws] + [AdditiveShare(last)])
        if reference_rng:
            bls = [v.bit_length() if bit_length is None else bit_length for v in values]
            rows = D.reference_share_draws(bls, num_shares - 1)
            last = _reconstruct([values] + [[-d for d in r] for r in rows])
            return AdditiveShares([AdditiveShare(r) for r in rows] + [AdditiveShare(last)])
        if _in_64bit_domain(values) and (bit_length is None or bit_length <= 64):
            unsigned = _device_domain(values)
            host = np.array([v if not unsigned or v < 2**63 else v - 2**64 for v in values], dtype=np.int64)
            sec = torch.from_numpy(host).to(D.device())
            shares = D.ass_split(sec, num_shares, bit_length, unsigned=unsigned)
            rows = [D.int128_to_ints(s) for s in shares.cpu().numpy()]
        else:  # wide limbs: e.g. the 2040-bit JL user key of the key setup
            bmax = max(abs(v).bit_length() for v in values) if bit_length is None else bit_length
            l_in = (max(abs(v).bit_length() for v in values) + 1 + 31) // 32 + 1
            l_out = max(l_in + 1, (bmax + (num_shares - 1).bit_length() + 2 + 31) // 32 + 1)
            sec = torch.from_numpy(D.ints_to_limbs_tc(values, l_in)).to(D.device())
            shares = D.ass_split_wide(sec, num_shares, l_out, bit_length)
            rows = [D.limbs_tc_to_ints(s) for s in shares.cpu().numpy()]
        if isinstance(self._secret, int):
            return AdditiveShares([AdditiveShare(r[0]) for r in rows])
        return AdditiveShares([AdditiveShare(r) for r in rows])

    # ---- device fast path ----------------------------------------------------------------------
    @staticmethod
    def split_tensor(secret: torch.Tensor, num_shares: int, bit_length: Optional[int] = None,
                     unsigned: bool = False, elem_offset: int = 0) -> torch.Tensor:
        """int64 tensor in HBM -> int64 [num_shares, n, 2] int128 shares (lo, hi) in HBM."""
        if num_shares <= 0:
            raise FedbiomedValueError("Number of shares must be greater than 0")
        return D.ass_split(secret, num_shares, bit_length, unsigned=unsigned, elem_offset=elem_offset)


class AdditiveShare:
    """One share (reference `_additive_ss.py:101-181`)."""

    def __init__(self, value: Union[int, List[int]]) -> None:
        if not (isinstance(value, int) or (isinstance(value, list) and all(isinstance(i, int) for i in value))):
            raise FedbiomedTypeError("AdditiveShare value must be an int or a list of int")
        self._value = value

    def __add__(self, other: "AdditiveShare") -> "AdditiveShare":
        if isinstance(other, AdditiveShare):
            if isinstance(self._value, int) and isinstance(other.value, int):
                return AdditiveShare(_reconstruct([[self._value], [other.value]])[0])
            if isinstance(self.value, list) and isinstance(other.value, list):
                return AdditiveShare(_reconstruct([self.value, other.value[: len(self._value)]]))
            raise FedbiomedTypeError("AdditiveShares must be of the same type")
        raise FedbiomedTypeError("Additive share can be summed to only another Additive share")

    def __radd__(self, other: Union[int, "AdditiveShare"]):
        if other == 0:
            return self
        return self.__add__(other)

    def __repr__(self) -> str:
        return f"AdditiveShare({self.value})"

    @property
    def value(self) -> Union[int, List[int]]:
        return self._value


def _reconstruct(rows: List[List[int]]) -> List[int]:
    """Exact column sum of equal-length int rows on the device: int128 lanes when the
    values and their sum fit, two's-complement u32 limbs of any width otherwise."""
    if not rows or not rows[0]:
        return []
    bits = max(abs(int(v)).bit_length() for r in rows for v in r)
    if bits + len(rows).bit_length() < 126:
        arr = np.stack([D.ints_to_int128(r) for r in rows])
        out = D.ass_reconstruct(torch.from_numpy(arr).to(D.device()))
        return D.int128_to_ints(out.cpu().numpy())
    L = (bits + len(rows).bit_length() + 2 + 31) // 32
    arr = np.stack([D.ints_to_limbs_tc(r, L) for r in rows])
    out = D.ass_reconstruct_wide(torch.from_numpy(arr).to(D.device()))
    return D.limbs_tc_to_ints(out.cpu().numpy())


class AdditiveShares(list):
    """Collection of shares (reference `_additive_ss.py:184-267`)."""

    def __init__(self, shares: List[AdditiveShare]) -> None:
        if not all(isinstance(share, AdditiveShare) for share in shares):
            raise FedbiomedTypeError("All shares must be of type Share")
        super().__init__(shares)

    def __add__(self, other: "AdditiveShares") -> "AdditiveShares":
        if len(self) != len(other):
            raise FedbiomedTypeError("AdditiveShares must be of the same length")
        if all(isinstance(share.value, int) for share in self) != all(isinstance(share.value, int) for share in other):
            raise FedbiomedTypeError("AdditiveShares must be of the same type")
        if all(isinstance(share.value, int) for share in self) or all(isinstance(share.value, list) for share in self):
            return AdditiveShares([self[i] + other[i] for i in range(len(self))])
        raise FedbiomedTypeError("AdditiveShares must be of the same type")

    def __radd__(self, other: Union[int, "AdditiveShares"]):
        if other == 0:
            return self
        return self.__add__(other)

    def to_list(self) -> List[Union[int, List[int]]]:
        return [share.value for share in self]

    def reconstruct(self) -> Union[int, List[int]]:
        if all(isinstance(share.value, int) for share in self):
            return _reconstruct([[share.value] for share in self])[0]
        if all(isinstance(share.value, list) for share in self):
            n = len(self[0].value)
            return _reconstruct([share.value[:n] for share in self])
        raise FedbiomedTypeError("Shares must be of the same type")

    @staticmethod
    def reconstruct_tensor(shares: torch.Tensor) -> torch.Tensor:
        """int64 [P, n, 2] int128 shares in HBM -> int64 [n, 2] exact sums in HBM."""
        return D.ass_reconstruct(shares)
