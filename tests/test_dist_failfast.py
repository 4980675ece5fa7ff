"""A failing rank ends the run: the process group's collectives time out after
distributed.pg_timeout() (FBM_DIST_TIMEOUT_S, default 120 s, not torch's 10 min for NCCL), and a rank
body run under distributed.run_rank exits non-zero as soon as it raises.  gloo, world size 2, CPU:
rank 1 raises before the first collective; rank 0 waits in an all-reduce.  Both processes must exit
non-zero well inside the timeout."""

import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

BODY = r"""
import os, sys
sys.path.insert(0, {root!r})
import torch
from fedbiomed_amd import distributed as Dd

def body():
    rank, world, _ = Dd.init("gloo")
    assert world == 2
    if rank == 1:
        raise RuntimeError("rank 1 fails before the collective")
    t = torch.ones(4)
    torch.distributed.all_reduce(t)  # waits for rank 1, which never comes
    print("rank 0 passed the collective", flush=True)

Dd.run_rank(body)
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_failing_rank_ends_both_ranks_within_the_timeout():
    timeout_s = 20
    port = _port()
    code = BODY.format(root=ROOT)
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FBM_DIST_TIMEOUT_S=str(timeout_s))
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout_s + 60)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a rank did not exit within the process group's timeout")
        outs.append((p.returncode, o, e))
    elapsed = time.time() - t0
    assert outs[1][0] != 0 and "rank 1 fails" in outs[1][2]
    assert outs[0][0] != 0, outs[0]
    assert "passed the collective" not in outs[0][1]
    assert elapsed < timeout_s + 45


def test_pg_timeout_default_and_env(monkeypatch):
    from fedbiomed_amd import distributed as Dd

    monkeypatch.delenv("FBM_DIST_TIMEOUT_S", raising=False)
    assert Dd.pg_timeout().total_seconds() == 120
    monkeypatch.setenv("FBM_DIST_TIMEOUT_S", "7.5")
    assert Dd.pg_timeout().total_seconds() == 7.5


BODY_STUCK = r"""
import os, sys, time
sys.path.insert(0, {root!r})
import torch
from fedbiomed_amd import distributed as Dd

def body():
    rank, world, _ = Dd.init("gloo")
    if rank == 1:
        time.sleep({sleep})  # alive but never joins: rank 0's collective must time out
        return
    t = torch.ones(4)
    torch.distributed.all_reduce(t)
    print("rank 0 passed the collective", flush=True)

Dd.run_rank(body)
"""


def test_stuck_peer_times_out():
    timeout_s = 6
    port = _port()
    code = BODY_STUCK.format(root=ROOT, sleep=timeout_s + 20)
    env0 = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(port), FBM_DIST_TIMEOUT_S=str(timeout_s))
    env1 = dict(env0, RANK="1", LOCAL_RANK="1")
    t0 = time.time()
    p0 = subprocess.Popen([sys.executable, "-c", code], env=env0, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    p1 = subprocess.Popen([sys.executable, "-c", code], env=env1, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        o, e = p0.communicate(timeout=timeout_s + 40)
        t_exit = time.time() - t0
    finally:
        p1.kill()
        p1.communicate()
    assert p0.returncode != 0 and "passed the collective" not in o
    assert t_exit < timeout_s + 30, t_exit
