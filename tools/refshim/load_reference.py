"""Import the reference Fed-BioMed secagg hot path from /root/reference (read-only).

Test tooling for `tools/gen_golden.py` ONLY (runs in the survey/build container, never
on the GPU box, never imported by the product package).  Recipe = SURVEY.md Appendix A:

* `gmpy2` / `cryptography` are absent from the image: the shims next to this file
  stand in, backed by the system libgmp / libcrypto the real packages wrap;
* `fedbiomed/common/secagg/__init__.py` imports `_dh` (ECDH via cryptography), which the
  shim does not provide, so the package module is pre-registered empty and only the
  hot-path submodules are imported;
* `SHARE_DIR` (`fedbiomed/common/utils/_config_utils.py:34-55`) needs a
  `share/fedbiomed` dir: a temp user base with a symlink to the reference's
  `envs/common/default_biprimes` satisfies it.
"""

import os
import site
import sys
import tempfile
import types

REF = os.environ.get("FBM_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    """Returns a namespace with the reference hot-path classes/functions."""
    if not os.path.isdir(os.path.join(REF, "fedbiomed")):
        raise RuntimeError(f"reference not found at {REF}")
    sys.dont_write_bytecode = True
    ub = os.path.join(tempfile.gettempdir(), "fbm_ref_userbase")
    dst = os.path.join(ub, "share", "fedbiomed", "envs", "common")
    os.makedirs(dst, exist_ok=True)
    link = os.path.join(dst, "default_biprimes")
    if not os.path.exists(link):
        os.symlink(os.path.join(REF, "envs", "common", "default_biprimes"), link)
    site.USER_BASE = ub
    for p in (HERE, REF):
        if p not in sys.path:
            sys.path.insert(0, p)
    import fedbiomed.common as common  # noqa: E402

    pkg = types.ModuleType("fedbiomed.common.secagg")
    pkg.__path__ = [os.path.join(REF, "fedbiomed", "common", "secagg")]
    sys.modules["fedbiomed.common.secagg"] = pkg
    common.secagg = pkg
    import importlib

    lom = importlib.import_module("fedbiomed.common.secagg._lom")
    jls = importlib.import_module("fedbiomed.common.secagg._jls")
    crypter = importlib.import_module("fedbiomed.common.secagg._secagg_crypter")
    ass = importlib.import_module("fedbiomed.common.secagg._additive_ss")
    for mod in (lom, jls, crypter, ass):
        for k in dir(mod):
            if not k.startswith("__"):
                setattr(pkg, k, getattr(mod, k))
    utils = importlib.import_module("fedbiomed.common.utils")
    constants = importlib.import_module("fedbiomed.common.constants")
    ns = types.SimpleNamespace(lom=lom, jls=jls, crypter=crypter, ass=ass, utils=utils,
                               constants=constants, pkg=pkg)
    return ns
