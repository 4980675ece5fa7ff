#!/usr/bin/env python3
"""Headline benchmark: secure-aggregation encrypt+aggregate throughput on MI355X.

Metric (BASELINE.json): "params/s secagg encrypt+aggregate (device-resident), 10M-elem
vector @1/8 GPU".  One step = every party encrypts its device-resident parameter vector
(Joye-Libert by default: quantise, weight, VES-pack, FDH, 2048-bit modexp) followed by one
aggregate (ciphertext product, server-key exponentiation, inverse, unmask, decode, average,
dequantise).  value = params processed by all ranks / wall time of K steps (max over ranks).

Scaling: element-range sharding (fedbiomed_amd/distributed.py).  Default "strong": ONE 10M-element
vector (config 4) is split into N stripes, one per GPU, each processed with its global offsets -- the
total work is fixed as N grows -- and the step ends with the split's final gather (an RCCL all-gather
of the float64 output stripes: every rank holds the whole averaged vector).  `--weak` gives every
rank its own --elements stripe instead.  `stages` reports T_enc (all P parties' encrypts),
T_agg (the aggregate alone: decryption factor + combine), P*N/T_enc and N/T_agg.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scheme jl|lom] [--elements 10000000]
                    [--parties 8] [--weak]

At N = 1 the line also carries `end_to_end` (SURVEY 8(f), rank 0 only, outside the headline's clock): the
same work from pinned host memory, the reference's list API (one node's encrypt at 1M / 10M, the
researcher's aggregate at 1M x 8 and at the metric size, JL and LOM list round trips), each also after the
extensions that issue a call's work ahead (`prepare_encrypt` / `prepare_aggregate`: the factors, the output
objects), and the msgpack wire legs; and `cpu_baseline` (the oracle on a bounded sample, one host core).

With --gpus N > 1 and no torch.distributed.run environment, bench.py starts the N rank
processes itself (before anything touches a GPU) and relays rank 0's line.
"""

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# The step runs the P + 1 exponentiations on P + 1 HIP streams; HIP maps streams onto FIFO
# hardware queues (4 per process by default), so with 4 queues at most 4 launches run at once
# and the rest wait behind them.  16 queues (set before the runtime starts; the pool allows up
# to 32): 1/8-stripe step 183-186 -> 168-175 ms, 10M step 1174-1176 -> 1155-1158 ms (A/B on one
# box, tools/ab_hwq.sh, profiles/archive/r2_hwq_ab.txt).  An explicit setting in the environment wins.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
ISA_MAD_TOPS_2400 = 256 * 4 * 16 * 2.4e9 / 1e12  # 39.3 T: quarter-rate v_mad_u64_u32 at 2.4 GHz
MAD_PEAK_TOPS = 36.48        # measured v_mad_u64_u32 peak, whole chip, best occupancy (tools/microbench/madpeak.hip,
                             # profiles/archive/r1_madpeak.txt: 35.3 T at 2 waves/SIMD, 36.5 T at 4)
# v_mad_u64_u32 per lane of one N-adic product modulo N^2 -- the square, the general product and
# the short-base product (tools/gen_nadic_asm.py) -- are read from the library (fbm_jl_mads), so the
# count always matches the engine that ran.


def products_per_exp(key: int):
    """(squarings, general products, short-base products) of one jl_exp_kernel ciphertext on the
    short path (every bench ciphertext: one FDH digest, a 1024-bit N -- fbm_jl.hip): left-to-right
    binary over |key| below its top bit, a short-base product per 1 bit, then the host constant C and
    the final product with nude / 1 (two general products)."""
    k = abs(key)
    if k == 0:  # h = 1: to-Montgomery and the final product
        return 0, 2, 0
    return k.bit_length() - 1, 2, bin(k).count("1") - 1


def mads_per_exp(key: int, mads: tuple) -> int:
    return sum(c * m for c, m in zip(products_per_exp(key), mads))


def committed_traffic(kernel: str, scheme: str, elements: int, n_ct=None):
    """(HBM bytes per launch of `kernel`, the profile file) from the committed rocprofv3 PMC summary
    of this workload -- same scheme and elements per GPU (JL: same ciphertexts per party) --
    (profiles/*_hbm_traffic.json, written by tools/prof_summary.py), else (None, None).  `kernel` is
    the launched kernel's exact name with its template arguments (e.g. "lom_aggregate_ws_kernel<2, 4,
    8>"): a profile of another kernel or of another instantiation never stands in for it.  Not
    measured in the run: a PMC pass needs its own rocprofv3 process."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        cfg = d.get("meta", {}).get("bench_config") or {}
        if (cfg.get("scheme") == scheme and cfg.get("elements_per_gpu") == elements
                and (scheme != "jl" or cfg.get("ciphertexts_per_party_per_gpu") == n_ct)):
            k = d.get("kernels", {}).get("fbm::" + kernel)  # the exact instantiation only
            if k is not None:
                return k["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


class GfxClockSampler:
    """Samples the GPU's graphics clock (amdsmi, read-only) on a thread while a region runs: the
    clock the VALU peak is quoted against.  Every failure leaves `mhz` empty (the line says so)."""

    def __init__(self, index: int, period_s: float = 0.02):
        self.index, self.period, self.mhz, self._stop, self._t, self.error = index, period_s, [], None, None, None

    def __enter__(self):
        import threading

        try:
            import amdsmi

            amdsmi.amdsmi_init()
            handle = amdsmi.amdsmi_get_processor_handles()[self.index]
            self._stop = threading.Event()

            def run():
                while not self._stop.is_set():
                    try:
                        self.mhz.append(float(amdsmi.amdsmi_get_clock_info(handle, amdsmi.AmdSmiClkType.GFX)["clk"]))
                    except Exception as e:  # noqa: BLE001
                        self.error = repr(e)
                        return
                    self._stop.wait(self.period)

            self._t = threading.Thread(target=run, daemon=True)
            self._t.start()
        except Exception as e:  # noqa: BLE001
            self.error = repr(e)
        return self

    def __exit__(self, *exc):
        if self._t is not None:
            self._stop.set()
            self._t.join(timeout=5)
        try:
            import amdsmi

            amdsmi.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass
        return False

    def summary(self):
        if not self.mhz:
            return {"samples": 0, "error": self.error}
        v = sorted(self.mhz)
        return {"samples": len(v), "median_mhz": v[len(v) // 2], "min_mhz": v[0], "max_mhz": v[-1]}


def quiet_clipping_warnings():
    """bench.py only: the product logs the reference's clipping warning on every encrypt that clips
    (_secagg_utils.py:189-204); the synthetic inputs clip on purpose, so after the first one the
    bench drops the repeats, keeping the driver's stderr tail readable.  Other records pass."""
    import logging

    class Once(logging.Filter):
        seen = False

        def filter(self, rec):
            if "exceeds clipping range" not in rec.getMessage():
                return True
            if Once.seen:
                return False
            Once.seen = True
            rec.msg = str(rec.msg) + " (bench.py: further clipping warnings of this process suppressed)"
            return True

    logging.getLogger("fedbiomed_amd").addFilter(Once())


XGMI_LINK_BPS = 153e9  # one xGMI link, one direction (7 per MI355X): the all-gather model of the scaling probe


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scheme", choices=["jl", "lom"], default="jl")
    ap.add_argument("--elements", "--n", dest="n", type=int, default=10_000_000,
                    help="elements in total (strong, the default) or per GPU (--weak)")
    ap.add_argument("--parties", type=int, default=8)
    ap.add_argument("--weak", action="store_true", help="every rank owns its own --elements stripe")
    ap.add_argument("--strong", action="store_true", help="(the default) split --elements over the ranks")
    ap.add_argument("--no-stages", action="store_true", help="skip the per-stage T_enc / T_agg timing")
    ap.add_argument("--cpu-sample", type=int, default=None, help="elements in the timed CPU-oracle sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lom-extra", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-to-host (H2D/D2H-inclusive) legs")
    ap.add_argument("--no-e2e-full-agg", action="store_true",
                    help="skip the researcher list-API aggregate at the full vector size")
    ap.add_argument("--e2e-list-n", type=int, default=1_000_000, help="elements for the list-API end-to-end leg")
    ap.add_argument("--no-factor-overlap", action="store_true",
                    help="JL: compute the decryption factor inside the aggregate (after the encrypts)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL, the real runs) or gloo (rehearsal)")
    ap.add_argument("--no-prologue-first", action="store_true",
                    help="JL: issue each party's encrypt whole (prologue and exponentiation back to back)")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams for the parties' encrypts (0 = one per party); the decryption factor has its own")
    ap.add_argument("--no-batch-exp", action="store_true",
                    help="JL: one exponentiation launch per party (+ the factor's) on its own stream instead of "
                         "one batched launch over all of them (D.jl_exp_batch)")
    ap.add_argument("--serial", action="store_true",
                    help="no per-party streams in the timed steps (rocprof passes: per-kernel times unconfounded)")
    ap.add_argument("--rccl-world1", action="store_true",
                    help="at --gpus 1: form a world-1 RCCL process group, so the step ends with the strong-scaling "
                         "gather over RCCL (all_gather_shards) as every rank of an N-GPU run does")
    ap.add_argument("--node-list-n", type=int, nargs="*", default=[1_000_000, 10_000_000],
                    help="elements of the per-node list-API encrypt legs (one party's SecaggCrypter.encrypt)")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """--gpus N without a torch.distributed.run environment: start the N rank processes here,
    before this process touches a GPU (it never initialises HIP), and wait for them.  A rank
    that fails ends the others (by PID) so no rank waits forever in a collective."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0:
                rc = rc or code
                for q in procs:
                    q.kill()
        time.sleep(0.2)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import torch

    from fedbiomed_amd import _device as D, _native, distributed, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter

    quiet_clipping_warnings()
    rank, world, local = distributed.env_rank()
    # more ranks than visible GPUs only happens in a rehearsal (--dist-backend gloo on a
    # one-GPU box): ranks then share devices round-robin
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        distributed.init(args.dist_backend, device=local)
    elif args.rccl_world1:  # one rank, an RCCL group all the same: the gather leg runs over RCCL
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                             timeout=distributed.pg_timeout())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    P, tau = args.parties, 1
    ids = W.node_ids(P)
    weights = [W.party_weight(p) for p in range(P)]
    total_w = sum(weights)
    es, cr = D.jl_slot(None, P)

    # ---- this rank's stripe (global element offset) ----
    strong = not args.weak
    if strong:
        align = cr if args.scheme == "jl" else 8
        lo, hi = distributed.shard_range(args.n, world, rank, align)
        n_total = args.n
    else:
        per = ((args.n + cr * 8 - 1) // (cr * 8)) * (cr * 8) if world > 1 else args.n
        lo, hi = rank * per, rank * per + args.n
        n_total = args.n * world
    n = hi - lo
    # synthetic device-resident inputs (float32 model vectors, SURVEY §8(d) recipe)
    xs = [torch.from_numpy(W.party_params(p + 1000 * rank, n)).to(dev) for p in range(P)]
    keys = [W.jl_user_key(p) for p in range(P)]
    sk0 = -sum(keys)
    jc, lc = SecaggCrypter(), SecaggLomCrypter(W.LOM_NONCE)
    secrets_ = [W.pairwise_secrets_for(u, ids) for u in ids]

    n_ct_step = (n + cr - 1) // cr
    # one HIP stream per party: the parties' encrypts are independent, so the tail round
    # of one exponentiation launch overlaps the next party's launch
    n_streams = args.streams if args.streams > 0 else P
    pool = [torch.cuda.Stream(device=dev) for _ in range(n_streams)]
    streams = [pool[p % n_streams] for p in range(P)]
    main = torch.cuda.current_stream(dev)

    # strong scaling over N > 1 ranks: the step ends with the element-range split's final gather
    # (SURVEY 8(e)), so every rank -- the researcher -- holds the whole averaged vector
    gather = strong and (world > 1 or args.rccl_world1)
    factor_stream = torch.cuda.Stream(device=dev)
    overlap_factor = not args.no_factor_overlap
    batch_exp = not args.no_batch_exp and not args.no_prologue_first

    def engine_ctx(mode):
        """--no-batch-exp (an A/B form): the step's P + 1 concurrent exponentiation launches fill the
        chip together, so they take the throughput engine (one lane per ciphertext) even when each
        alone would be small -- the test build's per-thread switch, so those steps run through it.  The
        default step needs none: its one batched launch is the one-lane kernel, and it runs the product
        library throughout."""
        import contextlib

        return D.jl_engine(mode) if not batch_exp else contextlib.nullcontext()

    # the parties' ciphertexts go straight into their rows of the [P, n_ct, 64] block the aggregate
    # takes (encrypt_tensor(out=...)): no stacking copy inside the step
    CT = torch.empty((P, n_ct_step, 64), dtype=torch.int32, device=dev) if args.scheme == "jl" else None

    def step_jl(serial=False):
        cts = [None] * P
        factor = None
        with D.deferred_checks(), engine_ctx("single"):
            if args.no_prologue_first:
                if overlap_factor:
                    f_s = main if serial else factor_stream
                    f_s.wait_stream(main)
                    with torch.cuda.stream(f_s):
                        factor = jc.decrypt_factor_tensor(tau, n_ct_step, sk0, W.BIPRIME0, ct_offset=lo // cr)
                for p in range(P):
                    s_p = main if serial else streams[p]
                    s_p.wait_stream(main)
                    with torch.cuda.stream(s_p):
                        cts[p] = jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=weights[p],
                                                   ct_offset=lo // cr, out=CT[p])
            else:
                # Kernel order: every prologue (the parties' pack / N*pt+1 / FDH, the factor's FDH),
                # then every exponentiation, then the factor's inverse.  A running exponentiation
                # holds every CU slot, and the hardware queues are FIFO across the streams mapped
                # onto them: a small kernel queued behind an exponentiation waits for CU slots and
                # holds back whatever follows it on its queue (seen in the kernel trace).
                pend = [None] * P
                for p in range(P):
                    s_p = main if serial else streams[p]
                    s_p.wait_stream(main)
                    with torch.cuda.stream(s_p):
                        pend[p] = jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=weights[p],
                                                    ct_offset=lo // cr, defer_exp=True, out=CT[p])
                f_s = main if serial else factor_stream
                if overlap_factor:
                    f_s.wait_stream(main)
                    with torch.cuda.stream(f_s):
                        pf = jc.decrypt_factor_tensor(tau, n_ct_step, sk0, W.BIPRIME0, ct_offset=lo // cr,
                                                      phased=True)
                if not serial:  # the exponentiations start once all prologues are done
                    for st in pool + [factor_stream]:
                        main.wait_stream(st)
                    for st in pool + [factor_stream]:
                        st.wait_stream(main)
                if batch_exp:
                    # one launch over every party's ciphertexts and the factor's, on `main` (the
                    # serialised profiling step too: it times the step's own kernel)
                    with D.jl_exp_batch(dev):
                        if overlap_factor:
                            pf.exponentiate()
                        for p in range(P):
                            cts[p] = pend[p].finish()
                    if overlap_factor:
                        factor = pf.finish()
                else:
                    if overlap_factor:
                        with torch.cuda.stream(f_s):
                            pf.exponentiate()
                    for p in range(P):
                        with torch.cuda.stream(main if serial else streams[p]):
                            cts[p] = pend[p].finish()
                    if overlap_factor:
                        with torch.cuda.stream(f_s):
                            factor = pf.finish()
        if not serial:
            for st in pool + [factor_stream]:
                main.wait_stream(st)
            if factor is not None:
                factor.record_stream(main)
        out = jc.aggregate_tensor(tau, CT, sk0, W.BIPRIME0, total_w, num_expected_params=n,
                                  ct_offset=lo // cr, decrypt_factor=factor)
        if gather:  # the split's final gather: the whole averaged vector on every rank (RCCL all-gather)
            out = distributed.all_gather_shards(out, n_total, cr)
        return out

    # LOM stripes are ChaCha20-block (8-element) aligned: with the JL stripe (ciphertext aligned)
    # as the main workload, the LOM leg takes its own 8-aligned split of the same vector
    if args.scheme == "jl" and strong and world > 1:
        lo_l, hi_l = distributed.shard_range(args.n, world, rank, 8)
        xs_l = [torch.from_numpy(W.party_params(p + 1000 * rank, hi_l - lo_l)).to(dev) for p in range(P)]
    else:
        lo_l, hi_l, xs_l = lo, hi, xs
    Y = (torch.empty((P, hi_l - lo_l), dtype=torch.int64, device=dev)
         if args.scheme == "lom" or not args.no_lom_extra else None)

    def step_lom(serial=False):
        # the parties' overflow-guard status words are checked once per step, after the aggregate
        # is queued behind the protects (no per-party sync, no idle GPU while the host reads them)
        with D.deferred_checks():
            for p, u in enumerate(ids):  # each party's masked vector straight into its row
                lc.encrypt_tensor(tau, u, xs_l[p], secrets_[p], ids, weight=weights[p], elem_offset=lo_l, out=Y[p])
            out = lc.aggregate_tensor(Y, total_w)
        return distributed.all_gather_shards(out, n_total, 8) if gather else out

    def lom_cold_aggregate(reps=5):
        """The LOM aggregate with its input evicted from the chip's caches: the protects, then a write of
        a scratch buffer twice the MALL's 256 MB (MI355X_MICROARCH.md), then the aggregate alone, timed by
        the test build's HIP events on its stream (median of `reps`).  Inside the step the aggregate reads
        rows the protects wrote microseconds earlier, up to 256 MB of them from the MALL: that warm figure
        can exceed what HBM alone streams."""
        scratch = torch.empty(512 * 2 ** 20 // 8, dtype=torch.int64, device=dev)

        def once():
            with D.deferred_checks():
                for p, u in enumerate(ids):
                    lc.encrypt_tensor(tau, u, xs_l[p], secrets_[p], ids, weight=weights[p], elem_offset=lo_l,
                                      out=Y[p])
            scratch.fill_(1)
            torch.cuda.synchronize()
            _native.prof_enable(True)
            lc.aggregate_tensor(Y, total_w)
            torch.cuda.synchronize()
            _native.prof_enable(False)
            return _native.prof_report().get("lom_aggregate", (0, 0.0))

        with _native.test_hooks():
            once()  # warm-up through the test build
            runs = [once() for _ in range(reps)]
        del scratch
        ms = sorted(t / c for c, t in runs if c)[len(runs) // 2] if all(c for c, _ in runs) else None
        ab1 = 8 * (P + 1) * (hi_l - lo_l)
        return {"ms": ms, "hbm_GBps": ab1 / (ms / 1000) / 1e9 if ms else None,
                "hbm_frac": ab1 / (ms / 1000) / 1e9 / HBM_PEAK_GBS if ms else None, "runs": reps,
                "kernel": D.lom_aggregate_kernel(P, Y),
                "note": "median of %d: protects, 512 MB scratch write (2x the MALL), then the aggregate alone "
                        "(HIP events on its stream); the warm figure is the aggregate inside the step" % reps}

    def timed(step, steps, warmup, prof=False):
        """prof=True: serialised launches (one stream) with per-kernel HIP events, so each
        event pair brackets exactly one kernel's execution (roofline durations).  The event timer
        is the test build's (include/fbm_secagg_test.h): a profiled step runs through it
        (_native.test_hooks: the same kernel objects, the C ABI compiled with the timer), after one
        warm-up step of its own there; the timed steps of `value` run the product library."""
        import contextlib

        with (_native.test_hooks() if prof else contextlib.nullcontext()):
            for _ in range(warmup + (1 if prof else 0)):
                step(serial=prof)
            if world > 1:
                torch.distributed.barrier()
            torch.cuda.synchronize()
            if prof:
                _native.prof_enable(True)
            t0 = time.perf_counter()
            for _ in range(steps):
                step(serial=prof)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if prof:
                _native.prof_enable(False)
            if world > 1:
                torch.distributed.barrier()
            el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
            if world > 1:
                torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
            return el.item(), (_native.prof_report() if prof else {})

    step = step_jl if args.scheme == "jl" else step_lom
    if args.serial:
        step = (lambda f: (lambda serial=False: f(serial=True)))(step)
    elapsed, _ = timed(step, args.steps, args.warmup)
    value = n_total * args.steps / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    # one extra serialised step for the per-kernel durations (not part of `value`)
    prof_steps = 1
    with GfxClockSampler(local) as clk_s:
        _, kprof = timed(step, prof_steps, 0, prof=True)
    clk = clk_s.summary()

    # ---- roofline of the dominant kernel, from the live per-kernel HIP events ----
    n_ct = (n + cr - 1) // cr
    if args.scheme == "jl":
        cnt, ms = kprof.get("jl_exp", (0, 0.0))
        # algorithmic bytes of the launch(es) timed: the P parties' encrypts (4N +
        # 256*#ct each) and the decryption factor's output (256*#ct) -- the exponentiation launch
        # carries every party's and the factor's ciphertexts; the aggregate's own bytes belong to
        # the combine kernel, not to this launch
        alg_bytes = prof_steps * (P * (4 * n + 256 * n_ct) + 256 * n_ct)
        mm = sum(sum(products_per_exp(k)) for k in keys) + sum(products_per_exp(sk0))
        lib = _native.load_test()  # the engine's multiply counts (include/fbm_secagg_test.h)
        mads_mul, mads_sq, mads_short = lib.fbm_jl_mads(0), lib.fbm_jl_mads(1), lib.fbm_jl_mads(2)
        mads_step = n_ct * sum(mads_per_exp(k, (mads_sq, mads_mul, mads_short)) for k in keys + [sk0])
        mads = prof_steps * mads_step
        # the step's exponentiation kernel: one batched launch over every party and the factor
        # (jl_exp_kernel<true>), or one launch each (<false>, --no-batch-exp)
        kname = "jl_exp_kernel<true>" if batch_exp else "jl_exp_kernel<false>"
    else:
        cnt, ms = kprof.get("lom_aggregate", (0, 0.0))
        alg_bytes = prof_steps * 8 * (P + 1) * n
        mads, kname = 0, D.lom_aggregate_kernel(P, Y)  # the instantiation the launch takes
    sec = ms / 1000.0 if ms > 0 else float("nan")
    achieved = alg_bytes / sec / 1e9 if ms > 0 else None
    traffic, traffic_src = committed_traffic(kname, args.scheme, n, n_ct)
    roof = {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "algorithmic_bytes_per_launch": alg_bytes / cnt if cnt else None,
            "traffic": traffic,
            "traffic_source": (f"{traffic_src}: rocprofv3 PMC pass of this workload (2*FETCH_SIZE + WRITE_SIZE per "
                               "launch, committed; a PMC pass needs its own profiler process, so it is looked up, "
                               "not measured in this run)") if traffic_src else None,
            "avg_launch_ms": (ms / cnt) if cnt else None, "launches": cnt}
    if args.scheme == "lom":
        roof["cold"] = lom_cold_aggregate()
    if args.scheme == "jl" and cnt:
        # the bytes this launch must move by the data layout (csrc/fbm_internal.hpp), beside SURVEY §8(d)'s
        # path-level figure above: per party ciphertext jl_nude_kernel's digit 1 (FBM_NUDE_ROWS - FBM_NUDE_D1 =
        # 36 rows of 4 B) and the compact H row (8 words) in, the 256-B row out; the factor's H row in, its row out
        io = prof_steps * (P * n_ct * (144 + 32 + 256) + n_ct * (32 + 256))
        roof["kernel_io_bytes_per_launch"] = io / cnt
        roof["traffic_over_kernel_io"] = (traffic / (io / cnt)) if traffic else None
    if args.scheme == "jl":
        roof["note"] = ("jl_exp_kernel moves ~1e-4 of the HBM roofline's bytes by construction: it is bound by "
                        "integer multiply issue (v_mad_u64_u32), reported in roofline_valu; one launch = every "
                        "party's and the decryption factor's exponentiations (batched)")
    line = {
        "metric": "params/s secagg encrypt+aggregate (device-resident), 10M-elem vector @1/8 GPU",
        "value": value, "unit": "params/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong" if strong else "weak",
        "vs_baseline": None, "dtype": "u32-limb bigint (JL) / u64 (LOM); f32 in, f64 out",
        "data": "synthetic (float32 N(0,0.05^2) + 0.1% +/-4.0 outliers per party; biprime0; random 2040-bit keys)",
        "config": {"workload": f"{'Joye-Libert' if args.scheme == 'jl' else 'LOM'} encrypt (all {P} parties) + "
                               f"aggregate, {n:,} elements per GPU", "scheme": args.scheme, "parties": P,
                   "elements_per_gpu": n, "elements_total": n_total, "ciphertexts_per_party_per_gpu":
                   n_ct if args.scheme == "jl" else None, "parallelism": f"element-range x{world}"},
        "roofline": roof,
        "kernels_ms": {k: {"launches": c, "total_ms": round(t, 3)} for k, (c, t) in sorted(kprof.items())},
    }
    if args.scheme == "jl" and cnt:
        ach = mads / sec / 1e12
        line["roofline_valu"] = {"bound": "int-valu (v_mad_u64_u32)", "achieved": ach, "peak": MAD_PEAK_TOPS,
                                 "unit": "T lane-mad/s", "frac": ach / MAD_PEAK_TOPS,
                                 "peak_provenance": {
                                     "measured_T": MAD_PEAK_TOPS,
                                     "measured_note": "tools/microbench/madpeak.hip, profiles/archive/r1_madpeak.txt: best "
                                                      "occupancy (4 waves/SIMD) ran at 1.78 GHz -- power-limited",
                                     "isa_quarter_rate_T_at_2400MHz": ISA_MAD_TOPS_2400,
                                     "frac_of_isa_2400": ach / ISA_MAD_TOPS_2400,
                                     "isa_note": "256 CU x 4 SIMD x 16 lanes x 2.4 GHz (v_mad_u64_u32 at a quarter of "
                                                 "the 64-lane issue rate)",
                                     "gfx_clock_during_launch": clk,
                                     "isa_T_at_observed_clock": (ISA_MAD_TOPS_2400 * clk["median_mhz"] / 2400.0
                                                                 if clk.get("median_mhz") else None)},
                                 "products_per_ct_step": mm,
                                 "step_achieved": mads_step / (ms_per_step / 1000) / 1e12,
                                 "step_frac": mads_step / (ms_per_step / 1000) / 1e12 / MAD_PEAK_TOPS,
                                 "mads_per_square": mads_sq, "mads_per_product": mads_mul,
                                 "mads_per_short_product": mads_short,
                                 "note": "executed v_mad_u64_u32 of the N-adic engine (per square / product / "
                                         "short-base product above; the short path: a squaring per key bit, a "
                                         "short product per 1 bit, two general products); "
                                         "achieved/frac: the step's jl_exp launch(es) in a serialised step (HIP "
                                         "events on the launch stream); step_*: the timed step (all kernels)"}

    # ---- per-stage times: T_enc = all P parties' encrypts as the step issues
    #      them, T_agg = the aggregate alone (decryption factor + combine, nothing overlapped);
    #      each the median of a few runs, max over ranks ----
    if not args.no_stages:
        def t_stage(fn, reps=3):
            fn()
            ts = []
            for _ in range(reps):
                if world > 1:
                    torch.distributed.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t = torch.tensor([sorted(ts)[len(ts) // 2]], dtype=torch.float64, device=dev)
            if world > 1:
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            return t.item()

        if args.scheme == "jl":
            def enc_all():
                cts = [None] * P
                with D.deferred_checks(), engine_ctx("single"):
                    pend = [None] * P
                    for p in range(P):
                        streams[p].wait_stream(main)
                        with torch.cuda.stream(streams[p]):
                            pend[p] = jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=weights[p],
                                                        ct_offset=lo // cr, defer_exp=True)
                    for st in pool:
                        main.wait_stream(st)
                    for st in pool:
                        st.wait_stream(main)
                    if batch_exp:
                        with D.jl_exp_batch(dev):
                            for p in range(P):
                                cts[p] = pend[p].finish()
                    else:
                        for p in range(P):
                            with torch.cuda.stream(streams[p]):
                                cts[p] = pend[p].finish()
                for st in pool:
                    main.wait_stream(st)
                for c in cts:
                    c.record_stream(main)
                return torch.stack(cts)

            cts_all = enc_all()

            def agg_alone(k=n_ct, ne=n):
                part = cts_all if k == n_ct else cts_all[:, :k].contiguous()
                return jc.aggregate_tensor(tau, part, sk0, W.BIPRIME0, total_w, num_expected_params=ne,
                                           ct_offset=lo // cr)

            t_enc, t_agg = t_stage(enc_all), t_stage(agg_alone)
            # the combine alone, its factor issued ahead (decrypt_factor_tensor / prepare_aggregate: the
            # researcher knows the round, key and size before the nodes reply)
            fac = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0, ct_offset=lo // cr)
            t_comb = t_stage(lambda: jc.aggregate_tensor(tau, cts_all, sk0, W.BIPRIME0, total_w, num_expected_params=n,
                                                         ct_offset=lo // cr, decrypt_factor=fac))
            del fac
        else:
            def enc_all():
                with D.deferred_checks():
                    for p, u in enumerate(ids):
                        lc.encrypt_tensor(tau, u, xs[p], secrets_[p], ids, weight=weights[p], elem_offset=lo,
                                          out=Y[p])

            t_enc = t_stage(enc_all)
            t_agg = t_stage(lambda: lc.aggregate_tensor(Y, total_w))
        line["stages"] = {"T_enc_ms": 1000 * t_enc, "T_agg_ms": 1000 * t_agg,
                          "enc_party_params_per_s": P * n_total / t_enc, "agg_params_per_s": n_total / t_agg,
                          "note": "T_enc: all parties' encrypts (one stream each), T_agg: one aggregate alone "
                                  "(decryption factor + combine); max over ranks; rates over elements_total"}
        if args.scheme == "jl":
            line["stages"]["T_combine_factor_ahead_ms"] = 1000 * t_comb
            line["stages"]["note"] += ("; T_combine_factor_ahead: the aggregate with its decryption factor "
                                       "computed beforehand (the factor's exponentiations off the critical path)")
        if gather:  # the step's final all-gather of the float64 output stripes, alone
            stripe = torch.zeros(n, dtype=torch.float64, device=dev)
            align = cr if args.scheme == "jl" else 8
            line["stages"]["T_gather_ms"] = 1000 * t_stage(
                lambda: distributed.all_gather_shards(stripe, n_total, align))
        if args.scheme == "jl" and world == 1:
            # strong-scaling probe of the aggregate step on this GPU: T_agg of the stripe rank 0 of a
            # 2-, 4- and 8-GPU split owns (its first ciphertexts: ciphertext k depends only on its
            # global index, and rank 0's stripe is the largest) against T_agg of the whole vector
            probe = {}
            for g in (2, 4, 8):
                hig = distributed.shard_range(n, g, 0, cr)[1]
                kg = (hig + cr - 1) // cr
                tg = t_stage(lambda kg=kg, hig=hig: agg_alone(kg, hig))
                # the split's final all-gather of the float64 output (8 bytes per element): each rank
                # receives the other (g - 1) stripes -- modelled, not measured (one GPU here), at the xGMI
                # link rate: over one link at a time (a single-channel ring, the conservative bound) and
                # over the g - 1 direct links in parallel (a fully connected 8-GPU node)
                gb = (g - 1) / g * 8 * n
                t_ring, t_direct = gb / XGMI_LINK_BPS, gb / ((g - 1) * XGMI_LINK_BPS)
                probe[f"n{g}"] = {"stripe_elements": hig, "stripe_ciphertexts": kg, "T_agg_stripe_ms": 1000 * tg,
                                  "engine": D.jl_engine_for(kg), "ratio_whole_over_stripe": t_agg / tg,
                                  "gather_bytes_per_rank": gb,
                                  "T_gather_model_ms": {"ring_one_link": 1000 * t_ring,
                                                        "direct_all_links": 1000 * t_direct},
                                  "ratio_with_gather": t_agg / (tg + t_ring),
                                  "ratio_with_gather_direct": t_agg / (tg + t_direct)}
            line["stages"]["agg_scaling_probe"] = dict(probe["n8"], curve=probe, note=(
                "T_agg(whole vector) / T_agg(rank 0's stripe of an N-GPU split) on one GPU, N = 2 / 4 / 8: the "
                "aggregate step's strong-scaling bound (north star: >= 6x at N = 8); top-level fields = N = 8. "
                "ratio_with_gather adds the split's all-gather of the float64 output to the stripe's time: "
                "gather_bytes_per_rank / the xGMI link rate (%.0f GB/s per link, 7 links per MI355X; one link at a "
                "time = the conservative bound; _direct: the g - 1 links in parallel)" % (XGMI_LINK_BPS / 1e9)))
        if args.scheme == "jl":
            del cts_all

    # ---- secondary: LOM at the same size (cheap), so both schemes are on record ----
    if args.scheme == "jl" and not args.no_lom_extra:
        k2 = max(args.steps, 10)
        el2, _ = timed(step_lom, k2, 2)  # the step as it runs
        _, kp2 = timed(step_lom, 1, 0, prof=True)  # one instrumented step: per-kernel durations
        c2, m2 = kp2.get("lom_aggregate", (0, 0.0))
        ab = c2 * 8 * (P + 1) * (hi_l - lo_l)
        lom_kname = D.lom_aggregate_kernel(P, Y)  # the instantiation the launch takes
        line["lom"] = {"value": n_total * k2 / el2, "unit": "params/s",
                       "ms_per_step": 1000 * el2 / k2,
                       "aggregate_kernel": lom_kname,
                       "aggregate_traffic": committed_traffic(lom_kname, "lom", hi_l - lo_l),
                       "aggregate_hbm_GBps": ab / (m2 / 1000) / 1e9 if m2 else None,
                       "aggregate_hbm_frac": (ab / (m2 / 1000) / 1e9) / HBM_PEAK_GBS if m2 else None,
                       "kernels_ms": {k: {"launches": c, "total_ms": round(t, 3)} for k, (c, t) in sorted(kp2.items())}}
        line["lom"]["aggregate_cold"] = lom_cold_aggregate()

    # ---- secondary, N > 1: party-per-rank LOM -- the north star's RCCL reduce of the masked sum.
    #      Rank r protects parties r, r + N, ... over the WHOLE vector (the concatenation of every
    #      rank's element-range stripe of them, so the result is comparable), sums them, and one
    #      reduce-scatter of the u64 sums over xGMI leaves it the masked total of its stripe; it
    #      averages + dequantises that stripe and all-gathers the float64 stripes.  The output is
    #      checked bit for bit against the element-range LOM leg's gathered vector. ----
    if args.scheme == "jl" and strong and world > 1 and not args.no_lom_extra and P % world == 0:
        mine = [p for p in range(P) if p % world == rank]
        bnd = [distributed.shard_range(args.n, world, r, 8) for r in range(world)]
        xs_pp = [torch.from_numpy(np.concatenate([W.party_params(p + 1000 * r, b - a) for r, (a, b) in
                                                  enumerate(bnd)])).to(dev) for p in mine]
        Ypp = torch.empty((len(mine), args.n), dtype=torch.int64, device=dev)

        def step_pp(serial=False):
            with D.deferred_checks():
                for i, p in enumerate(mine):
                    lc.encrypt_tensor(tau, ids[p], xs_pp[i], secrets_[p], ids, weight=weights[p], out=Ypp[i])
                _, local = D.lom_aggregate(Ypp, 1, want_out=False, want_sums=True)
            stripe = distributed.reduce_scatter_u64(local, args.n)
            return distributed.all_gather_stripes(lc.aggregate_tensor(stripe.view(1, -1), total_w), args.n, 8)

        k3 = max(args.steps, 10)
        try:  # a secondary leg: a failure (the same on every rank) is recorded, not fatal to the line
            el3, _ = timed(step_pp, k3, 2)
            same = torch.tensor([int(torch.equal(step_pp(), step_lom()))], device=dev)
            torch.distributed.all_reduce(same, op=torch.distributed.ReduceOp.MIN)
            line["lom_party_per_rank"] = {
                "value": n_total * k3 / el3, "unit": "params/s", "ms_per_step": 1000 * el3 / k3,
                "parties_per_rank": len(mine), "equals_element_range": bool(same.item()),
                "backend": args.dist_backend,
                "note": "each rank protects its parties over the whole vector, local u64 sum, reduce-scatter "
                        "(RCCL over xGMI) of the masked sums, per-stripe average + dequantise, all-gather; "
                        "bit-exact vs the element-range LOM leg's gathered vector"}
        except Exception as e:  # noqa: BLE001
            line["lom_party_per_rank"] = {"error": repr(e)}

    # ---- secondary, N > 1: party-per-rank JL -- rank r encrypts parties r*P/N .. (r+1)*P/N - 1 over
    #      the WHOLE vector (the concatenation of every rank's element-range stripe of them), one
    #      all-to-all of ciphertext stripes (RCCL over xGMI; the modular product is no RCCL reduction),
    #      the aggregate of its ciphertext stripe at its ct_offset, all-gather of the float64 stripes;
    #      checked bit for bit against the element-range JL step's gathered vector ----
    if args.scheme == "jl" and strong and world > 1 and not args.no_lom_extra and P % world == 0:
        ppr = P // world
        mine = list(range(rank * ppr, (rank + 1) * ppr))  # rank-major party blocks
        bnd = [distributed.shard_range(args.n, world, r, cr) for r in range(world)]
        xs_pj = [torch.from_numpy(np.concatenate([W.party_params(p + 1000 * r, b - a) for r, (a, b) in
                                                  enumerate(bnd)])).to(dev) for p in mine]
        n_ct_all = (args.n + cr - 1) // cr

        def step_pj(serial=False):
            with D.deferred_checks():  # the whole vector per party: the cost model's one-lane engine
                cts_mine = torch.stack([jc.encrypt_tensor(P, tau, xs_pj[i], keys[p], W.BIPRIME0, weight=weights[p])
                                        for i, p in enumerate(mine)])
            stripe, k0 = distributed.all_to_all_ciphertexts(cts_mine, ppr)
            e_lo, e_hi = min(k0 * cr, args.n), min((k0 + stripe.shape[1]) * cr, args.n)
            out = jc.aggregate_tensor(tau, stripe, sk0, W.BIPRIME0, total_w, num_expected_params=e_hi - e_lo,
                                      ct_offset=k0)
            return distributed.all_gather_stripes(out, args.n, cr)

        kj = max(2, min(args.steps, 3))
        try:  # a secondary leg: a failure (the same on every rank) is recorded, not fatal to the line
            elj, _ = timed(step_pj, kj, 1)
            same = torch.tensor([int(torch.equal(step_pj(), step_jl()))], device=dev)
            torch.distributed.all_reduce(same, op=torch.distributed.ReduceOp.MIN)
            line["jl_party_per_rank"] = {
                "value": n_total * kj / elj, "unit": "params/s", "ms_per_step": 1000 * elj / kj,
                "parties_per_rank": ppr, "ciphertexts_per_rank_encrypted": ppr * n_ct_all,
                "equals_element_range": bool(same.item()), "backend": args.dist_backend,
                "note": "each rank encrypts its parties over the whole vector, all-to-all of ciphertext stripes "
                        "(RCCL over xGMI), aggregate of its stripe, all-gather; bit-exact vs the element-range "
                        "JL step's gathered vector"}
        except Exception as e:  # noqa: BLE001
            line["jl_party_per_rank"] = {"error": repr(e)}

    # ---- end-to-end legs (host memory in, host memory out): never `value` ----
    if rank == 0 and world == 1 and args.scheme == "jl" and not args.no_e2e:
        # (a) pinned host float32 vectors -> H2D -> encrypt -> D2H ciphertext limbs (each party),
        #     H2D of all ciphertexts -> aggregate -> D2H float64: the PCIe-inclusive rate
        xs_h = [xs[p].cpu().pin_memory() for p in range(P)]
        ct_h = [torch.empty((n_ct, 64), dtype=torch.int32).pin_memory() for _ in range(P)]
        out_h = torch.empty(n, dtype=torch.float64).pin_memory()
        cts_in = torch.empty((P, n_ct, 64), dtype=torch.int32, device=dev)  # the researcher's received block

        def step_e2e():
            # as the device-resident step: one stream per party (H2D -> prologue), the decryption
            # factor's prologue on its own stream, then the exponentiations (one batched launch),
            # each party's D2H of its ciphertexts and, on the same stream once it has landed in host
            # memory, the researcher's H2D of them into its row of the received block (PCIe is full
            # duplex: party p's H2D runs beside party p + 1's D2H); then combine -> D2H
            with D.deferred_checks():
                pend = [None] * P
                for p in range(P):
                    streams[p].wait_stream(main)
                    with torch.cuda.stream(streams[p]):
                        x_d = xs_h[p].to(dev, non_blocking=True)
                        pend[p] = jc.encrypt_tensor(P, tau, x_d, keys[p], W.BIPRIME0, weight=weights[p],
                                                    defer_exp=True)
                factor_stream.wait_stream(main)
                with torch.cuda.stream(factor_stream):
                    pf = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0, phased=True)
                for st in pool + [factor_stream]:
                    main.wait_stream(st)
                for st in pool + [factor_stream]:
                    st.wait_stream(main)
                if batch_exp:  # one exponentiation launch on `main`, then each party's D2H on its stream
                    with D.jl_exp_batch(dev):
                        pf.exponentiate()
                        cts_d = [pend[p].finish() for p in range(P)]
                    factor = pf.finish()
                    for p in range(P):
                        streams[p].wait_stream(main)
                        with torch.cuda.stream(streams[p]):
                            ct_h[p].copy_(cts_d[p], non_blocking=True)
                            cts_d[p].record_stream(streams[p])
                            cts_in[p].copy_(ct_h[p], non_blocking=True)
                else:
                    with torch.cuda.stream(factor_stream):
                        pf.exponentiate()
                    for p in range(P):
                        with torch.cuda.stream(streams[p]):
                            ct_h[p].copy_(pend[p].finish(), non_blocking=True)
                            cts_in[p].copy_(ct_h[p], non_blocking=True)
                    with torch.cuda.stream(factor_stream):
                        factor = pf.finish()
            for st in pool + [factor_stream]:
                main.wait_stream(st)
            factor.record_stream(main)
            out_h.copy_(jc.aggregate_tensor(tau, cts_in, sk0, W.BIPRIME0, total_w, num_expected_params=n,
                                            decrypt_factor=factor), non_blocking=True)
            torch.cuda.synchronize()

        step_e2e()
        t0 = time.perf_counter()
        step_e2e()
        te = time.perf_counter() - t0
        # the round trip through host memory changes nothing: the researcher's block is the device step's
        # ciphertexts and the floats are the tensor aggregate's, bit for bit
        e2e_equal = bool(torch.equal(cts_in, CT)) and bool(torch.equal(
            out_h, D.to_host(jc.aggregate_tensor(tau, CT, sk0, W.BIPRIME0, total_w, num_expected_params=n))))
        # (b) the reference's list API (List[float] in, List[int] out per party; List[List[int]] in,
        #     List[float] out), on a bounded sample: Python int <-> limb conversion dominates
        nl = min(args.e2e_list_n, n)
        xl = [xs_h[p][:nl].tolist() for p in range(P)]
        t0 = time.perf_counter()
        cl = [jc.encrypt(P, tau, xl[p], keys[p], W.BIPRIME0, weight=weights[p]) for p in range(P)]
        agg_l = jc.aggregate(tau, P, cl, sk0, W.BIPRIME0, total_w, num_expected_params=nl)
        tl = time.perf_counter() - t0
        del agg_l  # (results are freed outside the clock: a caller keeps them)
        # the same with every call prepared (prepare_encrypt per party, prepare_aggregate -- extensions whose
        # exponentiations run while the nodes train: outside the clock, each followed by a sync)
        tlp, clp = 0.0, []
        for p in range(P):
            jc.prepare_encrypt(tau, P, keys[p], W.BIPRIME0, nl)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            clp.append(jc.encrypt(P, tau, xl[p], keys[p], W.BIPRIME0, weight=weights[p]))
            tlp += time.perf_counter() - t0
        jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, nl)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        agg_lp = jc.aggregate(tau, P, clp, sk0, W.BIPRIME0, total_w, num_expected_params=nl)
        tlp += time.perf_counter() - t0
        list_prepared_equal = clp == cl
        del agg_lp, clp

        # (b2) the per-node numbers a deployment sees: ONE party's SecaggCrypter.encrypt(List[float])
        #      -- the node's call (node/secagg/_secagg_round.py:142-157) -- at 1M and 10M elements, and
        #      the researcher's aggregate(List[List[int]]) of the P parties' lists at nl elements
        #      (researcher/secagg/_secure_aggregation.py:644-655), wall time split into the host
        #      conversions and the GPU
        def node_encrypt(ne):
            xl0 = xs_h[0][:ne].tolist()
            jc.encrypt(P, tau, xl0[:cr * 64], keys[0], W.BIPRIME0, weight=weights[0])  # warm the staging
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = jc.encrypt(P, tau, xl0, keys[0], W.BIPRIME0, weight=weights[0])
            t_tot = time.perf_counter() - t0
            # the same call after SecaggCrypter.prepare_encrypt (an extension: H(t_k)^key issued with the
            # training request, done while the node trains): one product per ciphertext instead of an
            # exponentiation
            prepared = jc.prepare_encrypt(tau, P, keys[0], W.BIPRIME0, ne)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r2 = jc.encrypt(P, tau, xl0, keys[0], W.BIPRIME0, weight=weights[0])
            t_prep = time.perf_counter() - t0
            same = r2 == r
            del r, r2
            # the same call in its parts: list -> pinned f64 -> device | encrypt kernels | D2H -> ints
            t0 = time.perf_counter()
            x_d = D.floats_to_host(xl0).to(dev)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ct_d = jc.encrypt_tensor(P, tau, x_d, keys[0], W.BIPRIME0, weight=weights[0])
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            r = D.limbs_to_ints(D.to_host(ct_d).numpy().view(np.uint32))
            t3 = time.perf_counter()
            del r
            return {"elements": ne, "ciphertexts": (ne + cr - 1) // cr, "ms": 1000 * t_tot, "params_per_s": ne / t_tot,
                    "host_in_ms": 1000 * (t1 - t0), "gpu_ms": 1000 * (t2 - t1), "host_out_ms": 1000 * (t3 - t2),
                    "engine": D.jl_engine_for((ne + cr - 1) // cr),
                    "factor_prepared": {"ms": 1000 * t_prep, "params_per_s": ne / t_prep, "prepared": prepared,
                                        "equals_unprepared": same}}

        node_legs = {str(ne): node_encrypt(ne) for ne in args.node_list_n if ne <= n}
        n2 = W.BIPRIME0 * W.BIPRIME0

        def researcher_aggregate(cl_u, ne, reps=1):
            """SecaggCrypter.aggregate(List[List[int]]) of the P parties' lists at ne elements, and the
            same call's two halves alone: the host conversion (ints -> pinned limbs -> H2D) and the GPU
            (aggregate_tensor + D2H + float list).  Best of `reps` calls."""
            nct_u = len(cl_u[0])
            t0 = time.perf_counter()
            staged = D.host_empty((P, nct_u, 64), torch.int32)
            limbs = staged.numpy().view(np.uint32)
            for u in range(P):
                D.ints_to_limbs(cl_u[u], n2, out=limbs[u])
            cts_u = staged.to(dev)
            torch.cuda.synchronize()
            t_conv = time.perf_counter() - t0
            t0 = time.perf_counter()
            ref_out = D.to_host(jc.aggregate_tensor(tau, cts_u, sk0, W.BIPRIME0, total_w,
                                                    num_expected_params=ne)).numpy().tolist()
            t_gpu = time.perf_counter() - t0
            del cts_u, staged
            best, res = None, None
            for _ in range(reps):
                res = None  # the previous call's list is freed outside the clock (10M floats: ~50 ms)
                t0 = time.perf_counter()
                res = jc.aggregate(tau, P, cl_u, sk0, W.BIPRIME0, total_w, num_expected_params=ne)
                t = time.perf_counter() - t0
                best = t if best is None else min(best, t)
            eq = res == ref_out
            # the same call after prepare_aggregate (the factor issued when the training request goes out,
            # done by the time the nodes reply: the synchronize stands for their training time)
            res = None
            prepared = jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, ne)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = jc.aggregate(tau, P, cl_u, sk0, W.BIPRIME0, total_w, num_expected_params=ne)
            tp = time.perf_counter() - t0
            return {"elements": ne, "parties": P, "ciphertexts_per_party": nct_u, "ms": 1000 * best,
                    "params_per_s": ne / best, "host_conversion_ms": 1000 * t_conv, "gpu_ms": 1000 * t_gpu,
                    "equals_tensor_api": eq,
                    "factor_prepared": {"ms": 1000 * tp, "params_per_s": ne / tp, "prepared": prepared,
                                        "equals_tensor_api": res == ref_out}}

        agg_l = researcher_aggregate(cl, nl)
        t_agg_l = agg_l["ms"] / 1000
        # at the metric's size: the P parties' lists of the step's own 10M-element ciphertexts (CT)
        agg_full = None
        if n > nl and not args.no_e2e_full_agg:
            cl_full = [D.limbs_to_ints(D.to_host(CT[p]).numpy().view(np.uint32)) for p in range(P)]
            agg_full = researcher_aggregate(cl_full, n, reps=2)
            del cl_full
        # (c) over the wire: the same updates through a msgpack Serializer configured as the
        #     reference's (strict_types, one {"__type__": "int"} map per big int) vs the
        #     EncryptedParams hook (one bin per update), encrypt -> dumps -> loads -> aggregate
        import math

        import msgpack

        from fedbiomed_amd import wire

        def ref_default(o):
            w = wire.to_wire(o)
            if w is not None:
                return w
            if isinstance(o, int):
                return {"__type__": "int", "value": o.to_bytes(math.ceil(o.bit_length() / 8) + 1, "big", signed=True)}
            raise TypeError(type(o))

        def ref_hook(o):
            o = wire.from_wire(o)
            if isinstance(o, dict) and o.get("__type__") == "int":
                return int.from_bytes(o["value"], "big", signed=True)
            return o

        def over_wire(updates):
            blobs = [msgpack.packb({"params": u}, default=ref_default, strict_types=True) for u in updates]
            recv = [msgpack.unpackb(b, object_hook=ref_hook, strict_map_key=False)["params"] for b in blobs]
            return recv, sum(len(b) for b in blobs)

        t0 = time.perf_counter()
        recv, ref_bytes = over_wire(cl)
        t_ref_ser = time.perf_counter() - t0
        del recv
        wire.enable()
        try:
            t0 = time.perf_counter()
            cw = [jc.encrypt(P, tau, xl[p], keys[p], W.BIPRIME0, weight=weights[p]) for p in range(P)]
            recv, wire_bytes = over_wire(cw)
            agg_w = jc.aggregate(tau, P, recv, sk0, W.BIPRIME0, total_w, num_expected_params=nl)
            tw = time.perf_counter() - t0
            del agg_w, recv
            t0 = time.perf_counter()
            recv_w = over_wire(cw)
            t_wire_ser = time.perf_counter() - t0
            del recv_w
        finally:
            wire.enable(False)

        def reassembly(nbytes):  # one message of nbytes in the transport's 4 MB chunks (constants.py:121)
            cut = 4000000 - 33
            msg = np.random.default_rng(9).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
            chunks = [msg[i:i + cut] for i in range(0, nbytes, cut)]
            k = len(chunks)
            t0 = time.perf_counter()
            reply = bytes()
            for c in chunks:  # the reference's loop (transport/server.py:236-239)
                reply += c
            t_ref = time.perf_counter() - t0
            asm = wire.ChunkAssembler()
            t0 = time.perf_counter()
            for it, c in enumerate(chunks, 1):
                out = asm.add(c, k, it)
            t_asm = time.perf_counter() - t0
            assert out == reply
            return {"bytes": nbytes, "chunks": k, "reference_ms": 1000 * t_ref, "chunk_assembler_ms": 1000 * t_asm}

        per_party = 10_000_000 / nl  # one party's update at the metric's 10M elements
        chunk_reassembly = {"reference_encoding": reassembly(int(ref_bytes / P * per_party)),
                            "encrypted_params_blob": reassembly(int(wire_bytes / P * per_party)),
                            "note": "one party's 10M-element update received in the transport's 4 MB chunks: "
                                    "reply += chunk (the reference) vs fedbiomed_amd.wire.ChunkAssembler "
                                    "(SURVEY 8(f)2), host only"}
        line["end_to_end"] = {
            "wire": {"elements": nl, "parties": P,
                     "reference_encoding": {"bytes": ref_bytes, "dumps_loads_ms": 1000 * t_ref_ser,
                                            "list_api_plus_wire_params_per_s": nl / (tl + t_ref_ser)},
                     "encrypted_params_blob": {"bytes": wire_bytes, "dumps_loads_ms": 1000 * t_wire_ser,
                                               "list_api_plus_wire_params_per_s": nl / tw},
                     "chunk_reassembly": chunk_reassembly,
                     "note": "P updates through msgpack (reference Serializer rules) and back, then aggregate; "
                             "blob = fedbiomed_amd.wire hook (SURVEY 8(f)2)"},
            "pinned_host_tensors": {"value": n / te, "unit": "params/s", "ms_per_step": 1000 * te,
                                    "elements": n, "equals_device_step": e2e_equal,
                                    "note": "per party stream H2D + encrypt + D2H, then that "
                                                           "party's H2D into the researcher's block (beside "
                                                           "the next party's D2H); factor stream; combine + D2H"},
            "list_api": {"value": nl / tl, "unit": "params/s", "ms_per_step": 1000 * tl, "elements": nl,
                         "prepared": {"value": nl / tlp, "ms_per_step": 1000 * tlp,
                                      "equals_unprepared": list_prepared_equal},
                         "note": "SecaggCrypter.encrypt (List[float] -> List[int]) x P + aggregate "
                                 "(List[List[int]] -> List[float]), the P parties issued one after another in "
                                 "one process (a simulation artefact: each node encrypts on its own GPU); "
                                 "prepared: every call after its prepare_encrypt / prepare_aggregate "
                                 "(extensions; their GPU work outside the clock, as while the nodes train)"},
            "node_encrypt_list_api": dict(node_legs, note=(
                "one party's SecaggCrypter.encrypt(List[float]) -> List[int] (the node's call); host_in = list -> "
                "pinned float64 -> H2D, gpu = the encrypt kernels, host_out = D2H + limbs -> Python ints; "
                "factor_prepared: the call after SecaggCrypter.prepare_encrypt (an extension: the node's H(t_k)^key "
                "issued with the training request, done while it trains)")),
            "researcher_aggregate_list_api": dict(
                agg_l, at_metric_size=agg_full,
                note="SecaggCrypter.aggregate(List[List[int]]) of the P parties' ciphertext lists (at_metric_size: "
                     "the step's own 10M-element ciphertexts as Python ints, best of 2 calls); host_conversion "
                     "= ints -> pinned limbs -> H2D alone, gpu = aggregate_tensor + D2H + float list alone; the "
                     "call itself issues the decryption factor before converting, so ms < the sum; "
                     "factor_prepared: the call after SecaggCrypter.prepare_aggregate (an extension: the "
                     "factor issued with the training request, done when the nodes reply)")}

        # (d) LOM from and to host memory: pinned float32 -> H2D -> protect -> D2H u64 rows (one
        #     stream per party), then H2D of the rows -> aggregate -> D2H float64; and the
        #     reference's list API (SecaggLomCrypter.encrypt x P + aggregate) on the same sample
        if Y is not None:
            yh = [torch.empty(n, dtype=torch.int64).pin_memory() for _ in range(P)]
            lout_h = torch.empty(n, dtype=torch.float64).pin_memory()
            y_in = torch.empty_like(Y)  # the researcher's received block

            def step_lom_e2e():
                # per party stream: H2D -> protect -> D2H of its masked row, then (once it is in host
                # memory) the researcher's H2D of it into its row of the received block, beside the
                # next party's D2H; then aggregate -> D2H
                with D.deferred_checks():
                    for p, u in enumerate(ids):
                        streams[p].wait_stream(main)
                        with torch.cuda.stream(streams[p]):
                            x_d = xs_h[p].to(dev, non_blocking=True)
                            lc.encrypt_tensor(tau, u, x_d, secrets_[p], ids, weight=weights[p], out=Y[p])
                            yh[p].copy_(Y[p], non_blocking=True)
                            y_in[p].copy_(yh[p], non_blocking=True)
                for st in pool:
                    main.wait_stream(st)
                lout_h.copy_(lc.aggregate_tensor(y_in, total_w), non_blocking=True)
                torch.cuda.synchronize()

            step_lom_e2e()
            k3 = 5
            t0 = time.perf_counter()
            for _ in range(k3):
                step_lom_e2e()
            tle = (time.perf_counter() - t0) / k3
            lom_e2e_equal = bool(torch.equal(y_in, Y)) and bool(torch.equal(
                lout_h, D.to_host(lc.aggregate_tensor(Y, total_w))))
            t0 = time.perf_counter()
            yl = [lc.encrypt(tau, u, xl[p], secrets_[p], ids, weight=weights[p]) for p, u in enumerate(ids)]
            agg_ll = lc.aggregate(yl, total_w)
            tll = time.perf_counter() - t0
            del agg_ll, yl
            # the same with the output lists made ahead (SecaggLomCrypter.prepare_encrypt per party before
            # its encrypt, prepare_aggregate before the aggregate -- extensions, issued outside the clock as
            # a node does with the training request and the researcher before the replies)
            tlp = 0.0
            yl = []
            for p, u in enumerate(ids):
                lc.prepare_encrypt(tau, u, nl)
                t0 = time.perf_counter()
                yl.append(lc.encrypt(tau, u, xl[p], secrets_[p], ids, weight=weights[p]))
                tlp += time.perf_counter() - t0
            lc.prepare_aggregate(nl)
            t0 = time.perf_counter()
            agg_lp = lc.aggregate(yl, total_w)
            tlp += time.perf_counter() - t0
            del agg_lp, yl

            def lom_node_encrypt(ne):  # one party's encrypt(List[float]) -> List[int], as the JL legs
                xl0 = xs_h[0][:ne].tolist()
                lc.encrypt(tau, ids[0], xl0[:4096], secrets_[0], ids, weight=weights[0])  # warm the staging
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = lc.encrypt(tau, ids[0], xl0, secrets_[0], ids, weight=weights[0])
                t_plain = time.perf_counter() - t0
                prepared = lc.prepare_encrypt(tau, ids[0], ne)
                t0 = time.perf_counter()
                r2 = lc.encrypt(tau, ids[0], xl0, secrets_[0], ids, weight=weights[0])
                t_prep = time.perf_counter() - t0
                same = r2 == r
                del r, r2
                return {"elements": ne, "ms": 1000 * t_plain, "params_per_s": ne / t_plain,
                        "output_prepared": {"ms": 1000 * t_prep, "params_per_s": ne / t_prep, "prepared": prepared,
                                            "equals_unprepared": same}}

            lom_node = {str(ne): lom_node_encrypt(ne) for ne in args.node_list_n if ne <= n}
            line["end_to_end"]["lom"] = {
                "pinned_host_tensors": {"value": n / tle, "unit": "params/s", "ms_per_step": 1000 * tle,
                                        "elements": n, "equals_device_step": lom_e2e_equal,
                                        "note": "per party stream H2D f32 + protect + D2H u64 + "
                                                               "H2D of the row into the researcher's block "
                                                               "(beside the next party's D2H); aggregate + D2H f64"},
                "list_api": {"value": nl / tll, "unit": "params/s", "ms_per_step": 1000 * tll, "elements": nl,
                             "output_prepared": {"value": nl / tlp, "ms_per_step": 1000 * tlp},
                             "note": "SecaggLomCrypter.encrypt (List[float] -> List[int]) x P + aggregate "
                                     "(List[List[int]] -> List[float]); output_prepared: the same with each "
                                     "output list's objects made ahead (prepare_encrypt / prepare_aggregate, "
                                     "extensions; outside the clock)"},
                "node_encrypt_list_api": dict(lom_node, note=(
                    "one party's SecaggLomCrypter.encrypt(List[float]) -> List[int]; output_prepared: after "
                    "prepare_encrypt (the output's int objects made ahead, their values written in place)"))}

    # ---- CPU baseline: the oracle (CPU restatement of the reference, GMP powm) on a bounded sample ----
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import secagg_oracle as O

        ns = args.cpu_sample or (30_000 if args.scheme == "jl" else 500_000)  # JL: ~12.5 s on one core
        xs_c = [[float(v) for v in W.party_params(p, ns)] for p in range(P)]
        t0 = time.perf_counter()
        if args.scheme == "jl":
            cts = [O.jl_encrypt(xs_c[p], tau, keys[p], W.BIPRIME0, P, weight=weights[p]) for p in range(P)]
            O.jl_crypter_aggregate(cts, tau, sk0, W.BIPRIME0, total_w, ns)
        else:
            non = O.lom_nonce(W.LOM_NONCE)
            ys = [O.lom_encrypt(xs_c[p], tau, u, secrets_[p], ids, non, weight=weights[p])
                  for p, u in enumerate(ids)]
            O.lom_crypter_aggregate(ys, total_w)
        tc = time.perf_counter() - t0
        try:
            avail = len(os.sched_getaffinity(0))  # the cores this process may run on
        except (AttributeError, OSError):
            avail = os.cpu_count() or 1
        quota = D.cgroup_cpu_quota()  # the CPU time it may use (a cgroup limit: the box's CPU share)
        share = D.host_cpu_share()
        line["cpu_baseline"] = {"value": ns / tc, "unit": "params/s", "cores": 1, "kind": "port",
                                "sample": f"{ns:,} elements x {P} parties, encrypt all + aggregate, "
                                          f"{tc:.1f} s on 1 host core (oracle/secagg_oracle.py; GMP mpz_powm "
                                          f"via ctypes as gmpy2 does)",
                                "host_cores": {"available": avail, "machine": os.cpu_count(),
                                               "cgroup_cpu_quota": quota, "share": share},
                                "ideal_all_cores": {
                                    "value": ns / tc * share, "unit": "params/s", "cores": share,
                                    "note": "the 1-core rate x the CPUs this process may use -- its affinity, capped by "
                                            "its cgroup CPU quota (SURVEY 8(d)): the reference is single-threaded; "
                                            "every ciphertext is independent, so this is the ceiling of a perfectly "
                                            "parallel CPU port on this box's share, not a measurement"}}
        cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")  # tools/calibrate_cpu.py
        if os.path.exists(cal):
            with open(cal) as fh:
                c = json.load(fh).get(args.scheme)
            if c:
                r = c["reference_over_oracle_time"]
                line["cpu_baseline"]["reference_equivalent"] = {
                    "value": ns / tc / r, "unit": "params/s",
                    "note": f"the reference crypter itself ran {r:.3f}x the oracle's time on this sample in the "
                            "build container (profiles/cpu_calibration.json); it cannot run on the GPU box"}
        line["gpu_over_cpu"] = value / (ns / tc)
    if args.rccl_world1:
        line["config"]["gather"] = "all_gather_shards over a world-1 RCCL group (--rccl-world1)"
    if rank == 0:
        print(json.dumps(line))
    if world > 1 or args.rccl_world1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from fedbiomed_amd import distributed as _dist_guard

        _dist_guard.run_rank(main)  # a rank that raises ends its process non-zero at once
    else:
        main()
