#!/usr/bin/env python3
"""Do distributed.py's "nccl" (= RCCL) branches run at world size 2?  Two ranks share cuda:0 (the
only GPU of a gpurun box): if RCCL accepts two ranks on one device, every collective of the path
(reduce_scatter_u64, all_gather_stripes, all_gather_shards, all_to_all_ciphertexts) runs on device
tensors and is checked against its meaning computed on the host from the ranks' seeded inputs; if
RCCL refuses the shared device, the refusal is what the probe reports.  One JSON line.

    python tools/rccl_world2_probe.py [--timeout 90] [--backend nccl|gloo]
"""
import argparse
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_I64, N_F64, N_CT, P_LOCAL = 1003, 1003, 37, 2


def _inputs(rank):
    import torch

    g = torch.Generator().manual_seed(100 + rank)
    local = torch.randint(-2**62, 2**62, (N_I64,), dtype=torch.int64, generator=g)
    f64 = torch.randn(N_F64, dtype=torch.float64, generator=g)
    cts = torch.randint(-2**31, 2**31 - 1, (P_LOCAL, N_CT, 64), dtype=torch.int32, generator=g)
    return local, f64, cts


def _worker(rank, port, backend, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0")
    try:
        import torch
        import torch.distributed as dist

        from fedbiomed_amd import distributed as Dd

        Dd.init(backend, device=0)
        dev = torch.device("cuda", 0) if backend == "nccl" else torch.device("cpu")
        local, f64, cts = (t.to(dev) for t in _inputs(rank))
        ones = torch.ones(4, device=dev)
        dist.all_reduce(ones)
        lo, hi = Dd.shard_range(N_F64, 2, rank, 30)
        out = {
            "all_reduce": ones.cpu().numpy(),
            "reduce_scatter_u64": Dd.reduce_scatter_u64(local, N_I64).cpu().numpy(),
            "all_gather_stripes": Dd.all_gather_stripes(f64[Dd.stripe_bounds(N_F64, 2, 8)[1][rank][0]:
                                                              Dd.stripe_bounds(N_F64, 2, 8)[1][rank][1]],
                                                          N_F64, 8).cpu().numpy(),
            "all_gather_shards": Dd.all_gather_shards(f64[lo:hi].contiguous(), N_F64, 30).cpu().numpy(),
        }
        stripe, k0 = Dd.all_to_all_ciphertexts(cts, P_LOCAL)
        out["all_to_all_ciphertexts"] = stripe.cpu().numpy()
        out["k0"] = k0
        if backend == "nccl":
            torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except BaseException as e:  # noqa: BLE001 -- reported by the parent
        q.put((rank, f"{type(e).__name__}: {e}"))


def _expected():
    ins = [_inputs(r) for r in range(2)]
    local = [i[0].numpy() for i in ins]
    f64 = [i[1].numpy() for i in ins]
    cts = [i[2].numpy() for i in ins]
    from fedbiomed_amd import distributed as Dd

    tot = (local[0].view(np.uint64) + local[1].view(np.uint64)).view(np.int64)  # mod 2^64
    per_rank = {}
    for r in range(2):
        _, b = Dd.stripe_bounds(N_I64, 2, 8)
        rs = tot[b[r][0]:b[r][1]]
        _, bs = Dd.stripe_bounds(N_F64, 2, 8)
        gathered = np.concatenate([f64[s][bs[s][0]:bs[s][1]] for s in range(2)])
        shards = np.concatenate([f64[s][slice(*Dd.shard_range(N_F64, 2, s, 30))] for s in range(2)])
        _, bc = Dd.stripe_bounds(N_CT, 2, 1)
        a2a = np.concatenate([cts[s][:, bc[r][0]:bc[r][1]] for s in range(2)], axis=0)
        per_rank[r] = {"all_reduce": np.full(4, 2.0, np.float32), "reduce_scatter_u64": rs,
                       "all_gather_stripes": gathered, "all_gather_shards": shards,
                       "all_to_all_ciphertexts": a2a, "k0": bc[r][0]}
    return per_rank


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--timeout", type=float, default=90.0)
    ap.add_argument("--backend", default="nccl", help="gloo: the same harness on CPU tensors (tests)")
    args = ap.parse_args()
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, args.backend, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(2):
            r, v = q.get(timeout=args.timeout)
            got[r] = v
    except Exception as e:  # noqa: BLE001
        got["parent"] = f"{type(e).__name__}: {e}"
    for p in procs:
        p.join(timeout=20)
        if p.is_alive():
            p.kill()
            p.join()
    res = {"world": 2, "device": "cuda:0 shared by both ranks" if args.backend == "nccl" else "cpu",
           "backend": args.backend}
    errors = {str(k): v for k, v in got.items() if isinstance(v, str)}
    if errors or len(got) < 2:
        res.update(ran=False, errors=errors, exit_codes=[p.exitcode for p in procs])
    else:
        exp = _expected()
        checks = {}
        for r in range(2):
            for k, e in exp[r].items():
                g = got[r][k]
                ok = (g == e) if k == "k0" else (g.dtype == e.dtype and g.shape == e.shape and
                                                  np.array_equal(g.view(np.uint8), e.view(np.uint8)))
                checks[f"rank{r}.{k}"] = bool(ok)
        res.update(ran=True, all_equal=all(checks.values()), checks=checks)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
