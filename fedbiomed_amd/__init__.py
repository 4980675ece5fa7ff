"""fedbiomed_amd -- MI355X-native secure-aggregation crypter for Fed-BioMed.

Drop-in for the reference's `fedbiomed.common.secagg` crypters (Joye-Libert and LOM) and the
`fedbiomed.common.utils` quantisation helpers, with all arithmetic in hand-written gfx950
HIP kernels behind the C ABI of `include/fbm_secagg.h`.
"""

__version__ = "0.1.0"
