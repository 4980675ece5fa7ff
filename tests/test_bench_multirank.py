"""bench.py's N > 1 path end to end on one GPU: the orchestration the driver's N-GPU runs take
(rank processes, barrier + max-over-ranks timing, the strong split and its final gather, the
party-per-rank LOM / JL legs checked bit for bit against the element-range step, one JSON line
from rank 0).  Two ranks share cuda:0 over gloo here (two RCCL ranks cannot share one device);
the RCCL collectives themselves run in test_distributed.py::test_rccl_collectives_world1, and the
bench's gather over a world-1 RCCL group below.  Reference semantics: SURVEY §8(e),
/root/reference/fedbiomed/common/secagg/_lom.py:177-192."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--elements", "300000", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-e2e"]


def _bench(args, timeout=110):
    """bench.py in a child process (this test process may hold the GPU; the child starts fresh)."""
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_ranks_gloo_one_gpu():
    d = _bench(["--gpus", "2", "--dist-backend", "gloo"] + SMALL)
    assert d["n_gpus"] == 2 and d["steps"] == 1 and d["scaling"] == "strong"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["elements_total"] == 300000
    for leg in ("lom_party_per_rank", "jl_party_per_rank"):
        assert d[leg]["equals_element_range"] is True, leg
    assert "cpu_baseline" not in d  # rank 0 at N = 1 only


@pytest.mark.gpu
def test_bench_rccl_world1_gather():
    d = _bench(["--rccl-world1", "--no-lom-extra"] + SMALL)
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["stages"]["T_gather_ms"] >= 0
