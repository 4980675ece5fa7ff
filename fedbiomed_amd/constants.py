"""Constants mirrored from the reference (fedbiomed/common/constants.py:350-362, :412, :437, :442)."""

from enum import Enum


class SAParameters:
    CLIPPING_RANGE: int = 3
    TARGET_RANGE: int = 2**13
    WEIGHT_RANGE: int = 2**17
    KEY_SIZE: int = 2048
    FA_CLIPPING_RANGE: int = 100_000_000_000_000  # 1e14
    FA_TARGET_RANGE: int = 2**55


class ErrorNumbers(Enum):
    FB417 = "FB417: secure aggregation error"
    FB624 = "FB624: Secure aggregation crypter error"
    FB629 = "FB629: Diffie-Hellman KA error"
