"""tools/rccl_world2_probe.py (two ranks on one device through every collective of distributed.py,
checked against the collectives' meaning on the host) run with gloo on CPU tensors: the harness the
GPU box runs with "nccl" is itself right.  CPU only."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_world2_probe_harness_on_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_world2_probe.py"), "--backend", "gloo",
                        "--timeout", "120"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ran"] and res["all_equal"], res
    assert len(res["checks"]) == 12
