"""SecaggCrypter.prepare_aggregate (an extension) without a GPU: nothing is prepared and nothing
raises -- aggregate itself then raises the no-device error, as it does without a preparation.
CPU only."""
import torch

from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter
from fedbiomed_amd.secagg._secagg_crypter import _prep_tag


def test_prepare_without_device_prepares_nothing():
    jc = SecaggCrypter()
    if torch.cuda.is_available():  # (the GPU behaviour is tests/test_crypter_api.py's)
        return
    assert jc.prepare_aggregate(3, 2, -5, 2**61 - 1, 100) is False
    assert getattr(jc, "_prepared", None) is None
    assert SecaggLomCrypter().prepare_aggregate(3, 2, -5, 2**61 - 1, 100) is False


def test_prep_tag_keeps_no_key_and_separates_arguments():
    a = _prep_tag(3, 4, -123456789, 97, None)
    assert len(a) == 32 and b"123456789" not in a
    assert a == _prep_tag(3, 4, -123456789, 97, 2**13)  # None = the default target range
    others = [_prep_tag(4, 4, -123456789, 97, None), _prep_tag(3, 5, -123456789, 97, None),
              _prep_tag(3, 4, -123456788, 97, None), _prep_tag(3, 4, -123456789, 101, None),
              _prep_tag(3, 4, -123456789, 97, 2**55)]
    assert len({a, *others}) == 6
    assert _prep_tag(3, 4, 2**100000, 97, None) is not None  # no decimal conversion of a huge key
    assert _prep_tag(3.0, 4, 5, 97, None) is None and _prep_tag(3, 4, 5, "97", None) is None


class _Ev:
    def __init__(self):
        self.waited = False

    def synchronize(self):
        self.waited = True


def test_capture_and_adopt_checks():
    """Status words of work issued ahead (capture_checks) are checked by the call that adopts them: inside
    its deferred_checks (at that context's exit) or at once without one -- a device error flag raises
    there, not in the early call."""
    import numpy as np
    import pytest

    from fedbiomed_amd import _device as D

    err = 2  # FBM_ERR_FDH_OVERFLOW (csrc/fbm_internal.hpp): the reference's OverflowError
    ok, bad = torch.zeros(4, dtype=torch.int32), torch.zeros(4, dtype=torch.int32)
    bad[D.FBM_STAT_ERRFLAGS] = err
    with D.capture_checks() as cap:
        D.deferred_checks._stack()[-1].append((ok, (0, None), _Ev()))
        D.deferred_checks._stack()[-1].append((bad, (0, None), _Ev()))
    assert len(cap.pending) == 2 and D.deferred_checks._stack() == []  # nothing checked, nothing raised
    D.adopt_checks(cap.pending[:1])  # no context: checked at once, waiting for its event
    assert cap.pending[0][2].waited
    with pytest.raises(OverflowError):
        D.adopt_checks(cap.pending[1:])
    with D.deferred_checks() as outer:  # inside a context: appended, raised at its exit only
        D.adopt_checks([(ok, (0, None), _Ev())])
        assert len(D.deferred_checks._stack()[-1]) == 1
        D.deferred_checks._stack()[-1].clear()  # (no device here to stack the words on)
    assert outer is not None and np.asarray(bad)[D.FBM_STAT_ERRFLAGS] == err


def test_lom_prepare_aggregate_makes_floats_only():
    """SecaggLomCrypter.prepare_aggregate(num_params) (an extension): the output's floats, host only;
    the Joye-Libert form of the call and bad sizes prepare nothing."""
    lc = SecaggLomCrypter()
    assert lc.prepare_aggregate(5) is True and lc._lom_agg_pool == [0.0] * 5
    assert lc.prepare_aggregate(num_params=3) is True and len(lc._lom_agg_pool) == 3
    for bad in ((0,), (-1,), (2.0,), (True,), (3, 2, -5, 2**61 - 1, 100)):
        assert lc.prepare_aggregate(*bad) is False and lc._lom_agg_pool is None, bad
    assert lc.prepare_encrypt(1, "n", 0) is False and lc._lom_enc_prep is None
