"""The generated assembly headers the library compiles (fedbiomed_amd/csrc/fbm_{nadic,quad,tri,mont}_asm.hpp)
are exactly what their generators emit now: the simulator and interval-proof tests check the generators'
instruction lists, so a header edited by hand -- or a generator changed without rerunning it -- would ship
code those tests never saw.  The generators run with their defaults (no FBM_GEN_* A/B switch set)."""

import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fedbiomed_amd", "csrc")

pytestmark = pytest.mark.skipif(any(k.startswith("FBM_GEN_") for k in os.environ),
                                reason="an FBM_GEN_* A/B switch is set: the generators emit a variant")


def _load(name):
    spec = importlib.util.spec_from_file_location(f"_hdr_{name}", os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _shipped(fn):
    with open(os.path.join(CSRC, fn)) as f:
        return f.read()


def test_group_engine_headers_match_generator():
    Q = _load("gen_quad_asm")
    for g, pfx, PFX, name, fn in ((Q.QUAD, "qa", "QA", "QUAD", "fbm_quad_asm.hpp"),
                                  (Q.TRI, "ta", "TA", "TRIPLE", "fbm_tri_asm.hpp")):
        hdr, _, _ = Q.header(g, pfx, PFX, name)
        assert hdr == _shipped(fn), f"{fn} is stale: run python tools/gen_quad_asm.py"


@pytest.mark.parametrize("gen, fn", [("gen_nadic_asm", "fbm_nadic_asm.hpp"), ("gen_mont_asm", "fbm_mont_asm.hpp")])
def test_header_matches_generator(gen, fn, tmp_path, capsys):
    mod = _load(gen)
    mod.OUT = str(tmp_path / fn)
    mod.main()
    with open(mod.OUT) as f:
        assert f.read() == _shipped(fn), f"{fn} is stale: run python tools/{gen}.py"
