"""Mirrors of the reference's secagg utilities (fedbiomed/common/utils/_secagg_utils.py:82-187):
`quantize` and `reverse_quantize` run on the GPU (the LOM protect kernel with no peers is exactly
quantize; `fbm_dequantize` is reverse_quantize).  `multiply` / `divide` are generic arithmetic
helpers on any Python numbers (the reference's own tests call them on floats), kept as the
reference's list comprehensions: no secagg path calls them -- the crypters' weighting and averaging
are fused into their kernels, and `SecaggCrypter._apply_weighting` / `_apply_average` run on the
device (`fbm_int_ops`).
"""

from typing import List, Union

import numpy as np

from .. import _device as D
from ..constants import ErrorNumbers, SAParameters
from ..exceptions import FedbiomedSecaggCrypterError


def quantize(weights: List[float], clipping_range: Union[int, None] = None,
             target_range: int = SAParameters.TARGET_RANGE) -> List[int]:
    """q = uint64(min(T-1, (median(-c, x, c) + c) * T / (2c)))  -- in [0, T-1]."""
    D.quant_params(clipping_range, target_range)
    if len(weights) == 0:
        return []
    dev = D.device()
    x = D.floats_to_device([float(w) for w in weights], dev)
    y = D.lom_protect(x, [], [], b"\0" * 16, 0, 0, clip=clipping_range, target=target_range, weight=1)
    return D.u64_from_device(y)


def multiply(xs: List[int], k: int) -> List[int]:
    """reference _secagg_utils.py:122-134"""
    return [e * k for e in xs]


def divide(xs: List[int], k: int) -> List[float]:
    """reference _secagg_utils.py:137-149"""
    return [e / k for e in xs]


def reverse_quantize(weights: List[float], clipping_range: Union[int, None] = None,
                     target_range: int = SAParameters.TARGET_RANGE) -> List[float]:
    """-c + (2c)/(T-1) * float64(uint64(w)) for each w (values truncated to uint64 first)."""
    max_val = np.iinfo(np.uint64).max
    if any([v > max_val or v < 0 for v in weights]):
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: Cannot reverse quantize, received values exceed maximum number")
    D.dequant_params(clipping_range, target_range)  # ZeroDivisionError for T == 1, as the reference
    if len(weights) == 0:
        return []
    u = np.array(weights, dtype=np.uint64)  # the reference's truncating conversion
    dev = D.device()
    import torch

    ut = torch.from_numpy(u.view(np.int64)).to(dev)
    return D.dequantize(ut, clipping_range, target_range).cpu().numpy().tolist()
