"""FDH(2048, M).H(t_k) as two kernels (round 4): `jl_fdh_kernel` keeps the first digest when it is coprime
to M (every ciphertext of a real biprime) and marks the others, which `jl_fdh_retry_kernel` redoes with r
of up to 7 digests (reference `_jls.py:742-762`).  Moduli with small factors send many ciphertexts down the
retry path; each row is compared with the oracle's restatement (`oracle.secagg_oracle.fdh_bits`, pinned by
tests/golden/fdh_bits.json), over `ct_offset` ranges, and a ciphertext whose r never becomes coprime within
7 digests raises the reference's OverflowError."""

import pytest

from oracle import secagg_oracle as O

TAU = 7


def _oracle_rows(m, k0, k1):
    """k -> r (or None where the reference raises OverflowError)."""
    out = {}
    for k in range(k0, k1):
        try:
            out[k] = O.fdh_bits((k << 512) | TAU, m, 2048)
        except OverflowError:
            out[k] = None
    return out


def test_oracle_retry_rates():
    """The chosen moduli exercise both kernels: 1001^2 sends a quarter of the first digests to the retry
    path without any overflow; (2 N)^2 needs odd digests and overflows now and then."""
    odd = _oracle_rows(1001 ** 2, 0, 1000)
    assert all(r is not None for r in odd.values())
    assert 200 < sum(r.bit_length() > 256 for r in odd.values()) < 350


@pytest.mark.gpu
@pytest.mark.parametrize("m_kind", ["small_odd", "even_biprime", "biprime"])
def test_fdh_first_digest_and_retries_vs_oracle(m_kind):
    import torch

    from fedbiomed_amd import _device as D, workload as W

    n = 1000 if m_kind != "even_biprime" else 300
    m = {"small_odd": 1001 ** 2, "even_biprime": (2 * W.BIPRIME0) ** 2, "biprime": W.BIPRIME0 ** 2}[m_kind]
    want = _oracle_rows(m, 0, n)
    # contiguous runs of ciphertexts the reference hashes, each through its own ct_offset call
    runs, start = [], None
    for k in range(n + 1):
        ok = k < n and want[k] is not None
        if ok and start is None:
            start = k
        if not ok and start is not None:
            runs.append((start, k))
            start = None
    assert sum(b - a for a, b in runs) >= n - 10
    for a, b in runs:
        h = D.jl_fdh(b - a, m, TAU, ct_offset=a)
        torch.cuda.synchronize()
        got = D.limbs_to_ints(h.cpu().numpy().view("uint32"))
        for j, k in enumerate(range(a, b)):
            assert got[j] == want[k], (m_kind, k)
    for k in [k for k, r in want.items() if r is None][:3]:  # the reference's OverflowError, alone
        with pytest.raises(OverflowError, match="int too big to convert"):
            D.jl_fdh(1, m, TAU, ct_offset=k)
