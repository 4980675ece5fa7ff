"""The drop-in raises the reference's own exception classes when Fed-BioMed is importable.

Reference: fedbiomed/common/exceptions.py:10 (FedbiomedError), :209 (FedbiomedSecaggError),
:217 (FedbiomedSecaggCrypterError), :290, :306; the researcher routes on the base class,
researcher/federated_workflows/_federated_workflow.py:94 (`except FedbiomedError`).

A stub `fedbiomed/common/exceptions.py` (same hierarchy, same names) goes on sys.path of a fresh
interpreter; the crypters, the LOM class and DHKey must then raise instances of the stub's classes,
with no rebinding after import.  CPU only: every case fails in argument checks before any device
call."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_STUB = '''
class FedbiomedError(Exception):
    pass
class FedbiomedSecaggError(FedbiomedError):
    pass
class FedbiomedSecaggCrypterError(FedbiomedError):
    pass
class FedbiomedTypeError(FedbiomedError, TypeError):
    pass
class FedbiomedValueError(FedbiomedError, ValueError):
    pass
STUB_MARK = "stub"
'''

_SCRIPT = r'''
import sys
sys.path[:0] = [{stub!r}, {root!r}]
import fedbiomed.common.exceptions as F
from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter, DHKey
import fedbiomed_amd.exceptions as E
from fedbiomed_amd.secagg import _secagg_crypter, _jls, _dh
from fedbiomed_amd.utils import _secagg_utils
assert E.BOUND_TO_REFERENCE
for mod in (E, _secagg_crypter, _jls, _dh, _secagg_utils):
    cls = getattr(mod, "FedbiomedSecaggCrypterError", None)
    assert cls is None or cls is F.FedbiomedSecaggCrypterError, mod

def raised(fn):
    try:
        fn()
    except BaseException as e:  # noqa: BLE001
        return e
    raise AssertionError("no exception")

cases = {{
    "jl_int_params": lambda: SecaggCrypter().encrypt(num_nodes=2, current_round=1, params=[1], key=3,
                                                    biprime=1000000007 * 998244353),
    "jl_bad_num_nodes": lambda: SecaggCrypter().encrypt(num_nodes=-2, current_round=1, params=[0.5], key=3,
                                                       biprime=1000000007 * 998244353),
    "lom_bad_weight": lambda: SecaggLomCrypter(nonce="n").encrypt(current_round=1, node_id="a", params=[0.5],
                                                                 pairwise_secrets={{"b": b"k" * 32}},
                                                                 node_ids=["a", "b"], weight=2 ** 20),
    "jl_aggregate_count": lambda: SecaggCrypter().aggregate(current_round=1, num_nodes=3, params=[[1], [2]],
                                                           key=3, biprime=15, total_sample_size=2),
    "dh_bad_pem": lambda: DHKey(private_key_pem=b"-----BEGIN PRIVATE KEY-----\nnot a key\n"),
}}
for name, fn in cases.items():
    e = raised(fn)
    assert type(e) is F.FedbiomedSecaggCrypterError, (name, type(e), e)
    assert isinstance(e, F.FedbiomedError), name
    print(name, "OK", str(e)[:60])
'''


def _run(tmp_path, script):
    pkg = tmp_path / "fedbiomed" / "common"
    pkg.mkdir(parents=True)
    (tmp_path / "fedbiomed" / "__init__.py").write_text("")
    (pkg / "__init__.py").write_text("")
    (pkg / "exceptions.py").write_text(_STUB)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    return subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)


def test_reference_exception_classes_are_raised(tmp_path):
    r = _run(tmp_path, _SCRIPT.format(stub=str(tmp_path), root=ROOT))
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("jl_int_params", "jl_bad_num_nodes", "lom_bad_weight", "jl_aggregate_count", "dh_bad_pem"):
        assert f"{name} OK" in r.stdout


def test_mirrors_without_fedbiomed():
    code = textwrap.dedent(f"""
        import sys; sys.path.insert(0, {ROOT!r})
        import fedbiomed_amd.exceptions as E
        assert not E.BOUND_TO_REFERENCE
        assert issubclass(E.FedbiomedSecaggCrypterError, E.FedbiomedError)
        assert issubclass(E.FedbiomedTypeError, TypeError) and issubclass(E.FedbiomedValueError, ValueError)
        print("mirrors OK")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mirrors OK" in r.stdout, r.stdout + r.stderr
