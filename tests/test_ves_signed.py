"""VES.encode of negative values and of slots wider than their plaintext (round 5; the last two object-API
refusals of round 4's VES).  The reference ORs value j in at bit es j (_jls.py:169-176): a negative value makes
its plaintext Python's negative OR; with comp_ratio 0 its `bs` never reaches 0 (_jls.py:129-141), so one
plaintext holds every value, and decode reads min(v_expected, 0) = 0 values per plaintext (_jls.py:146-167).
On the device: fbm_ves_pack with is_signed (ABI 4: two's-complement rows whose sign extends to the top of the
plaintext).  JoyeLibert.protect / aggregate of such inputs take the reference's two steps, each on the device.
Fixture: tests/golden/ves_signed.json (tools/gen_golden.py gen_ves_signed, the reference's outputs)."""

import pytest

from oracle import secagg_oracle as O
from tests.golden_util import I, load


@pytest.fixture(scope="module")
def vs():
    return load("ves_signed.json")


def test_ves_signed_oracle_vs_fixture(vs):
    for c in vs["ves"]:
        V = [I(v) for v in c["V"]]
        E = [I(e) for e in c["E"]["ok"]]
        assert O.ves_encode(V, c["es"], c["cr"]) == E, (c["ptsize"], c["valuesize"], len(V))
        for d in c["decode"]:
            assert O.ves_decode(E, c["es"], c["cr"], d["v_expected"]) == [I(v) for v in d["out"]["ok"]]


def test_fixture_covers_the_refused_shapes(vs):
    assert any(c["cr"] == 0 for c in vs["ves"])
    assert any(min(I(v) for v in c["V"]) < 0 and c["cr"] > 1 for c in vs["ves"])
    assert any(I(p["target"]) > 2 ** 1024 for p in vs["protect"])


@pytest.mark.gpu
def test_ves_signed_device_vs_fixture(vs):
    from fedbiomed_amd.secagg._jls import VES

    for c in vs["ves"]:
        ves = VES(c["ptsize"], c["valuesize"])
        V, E = [I(v) for v in c["V"]], [I(e) for e in c["E"]["ok"]]
        assert ves.encode(V, c["add_ops"]) == E, (c["ptsize"], c["valuesize"], len(V))
        for d in c["decode"]:
            assert ves.decode(E, c["add_ops"], d["v_expected"]) == [I(v) for v in d["out"]["ok"]], d["v_expected"]


@pytest.mark.gpu
def test_joye_libert_negative_and_wide_slot_flows(vs):
    from fedbiomed_amd.secagg._jls import EncryptedNumber, JoyeLibert, ServerKey, UserKey
    from tests.test_jls_api import pp_of

    for p in vs["protect"]:
        n = I(p["n"])
        pp = pp_of(n)
        jl = JoyeLibert(target_range=I(p["target"]))
        rows = []
        for k, x, want in zip(p["keys"], p["xs"], p["cts"]):
            got = jl.protect(pp, UserKey(pp, I(k)), p["tau"], [I(v) for v in x], 3)
            assert got == [I(c) for c in want["ok"]]
            rows.append([EncryptedNumber(pp, c) for c in got])
        out = jl.aggregate(ServerKey(pp, I(p["sk0"])), p["tau"], rows, len(p["xs"][0]))
        assert out == [I(v) for v in p["aggregate"]["ok"]]
