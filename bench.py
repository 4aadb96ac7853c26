#!/usr/bin/env python3
"""Headline benchmark: RCCL all-reduce bus bandwidth on the scheduler-chosen k-GPU subset.

BASELINE.json metric: "RCCL all-reduce bus GB/s on scheduler-chosen k-GPU subset, k=1/2/4/8".

    python bench.py --gpus N --steps K --warmup W          # N=1 runs in-process
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One *step* = one out-of-place RCCL all-reduce (bf16, sum) of ``--size-mb`` MiB per GPU over the
subset the placement core picked from the node's discovered xGMI topology (rank r runs on
``subset[r]``).  Exactly K steps are timed between barrier + ``torch.cuda.synchronize()`` on both
sides; the max over ranks is reported.  ``busbw_gbps`` is the per-rank busBW = algBW * 2(k-1)/k
(nccl-tests convention); ``value`` is the whole-job aggregate the bench contract asks for, the
busBW of all k ranks summed (k * busbw_gbps) for k >= 2.  At k = 1 busBW is 0 by definition, so
``value`` is the algBW of the single-rank RCCL all-reduce (BASELINE.md "k=1 reports algBW only").  Per-GPU message size is fixed
as N grows ("weak" scaling).  Data is synthetic (exactly checked once before timing).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

METRIC = "RCCL all-reduce bus GB/s on scheduler-chosen k-GPU subset, k=1/2/4/8"

# (minCTAs, maxCTAs) of ncclConfig_t tried by the tuning pass; (0, 0) = RCCL's own channel count.
# A k-subset of the xGMI full mesh has k-1 links per GPU; more channels put more rings/CTAs on
# them, and which count saturates the links depends on k, so it is measured on the node.
TUNE_CANDIDATES = [(0, 0), (32, 128), (64, 128), (112, 128)]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size-mb", type=float, default=2048.0, help="per-GPU message size in MiB (default 2 GiB)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--backend", default="native", choices=["native", "torch", "cpu"],
                    help="native = RCCL communicator from csrc/rccl; torch = dist.all_reduce; cpu = gloo (control-path tests)")
    ap.add_argument("--inplace", action="store_true")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="small-message latency of hipGraph-captured vs eager all-reduces after the sweep "
                         "(auto = only at k = 1, where it has been run on MI355X; k >= 2 capture is opt-in)")
    ap.add_argument("--probe", default="auto", choices=["auto", "off", "quick", "full"],
                    help="HIP link probe (K4 warm-up + K1 p2p read of every ordered pair) before placement, in a child "
                         "process of rank 0; 'auto' = quick on GPUs, off for --backend cpu; a failed probe falls back "
                         "to the discovered link classes")
    ap.add_argument("--discovery", default="auto", choices=["auto", "amdsmi", "sysfs", "fake"])
    ap.add_argument("--cpu-visible", type=int, default=0,
                    help="--backend cpu: devices the job may place on (default: one per rank); e.g. 8 rehearses an "
                         "N<8 job on a whole 8-GPU node")
    ap.add_argument("--via", default="k8s", choices=["k8s", "direct"],
                    help="k8s = place the k-GPU pod through device plugin (gRPC) + extender (HTTP) + kubelet Allocate "
                         "in process; direct = call the placement core")
    ap.add_argument("--ctas", default="auto",
                    help="RCCL channel (CTA) bounds of the measured communicator: 'auto' = short tuning pass over "
                         f"{TUNE_CANDIDATES} at k >= 2 (untimed, before warmup), 'tune' = that pass at any k, "
                         "'default' = RCCL's choice, or MIN[:MAX]")
    ap.add_argument("--tune-steps", type=int, default=3, help="timed all-reduces per candidate in the tuning pass")
    ap.add_argument("--ab-worst", default="auto", choices=["auto", "on", "off"],
                    help="after the headline: time the same all-reduce on the WORST k-subset the placement core found "
                         "(a second communicator on those devices) and report the placement gain; auto = whenever a "
                         "distinct worst subset exists (k < devices on the node)")
    ap.add_argument("--ab-default", default="auto", choices=["auto", "on", "off"],
                    help="after the headline: also time the k-subset the kubelet hands out with no extender (lowest "
                         "free indices; the paper's default-Kubernetes comparator, p.7 Figs. 11-12) when it differs "
                         "from the chosen one")
    ap.add_argument("--topology-json", default="",
                    help="place on this node model (Topology JSON, e.g. a fixture with a degraded link) instead of "
                         "discovering one: rehearsals of the placement A/B on CPU")
    ap.add_argument("--rccl-log", default="auto", choices=["auto", "on", "off"],
                    help="capture RCCL's INIT/GRAPH log (per-rank file under /tmp) and report the transports and "
                         "channel counts it chose; auto = on for k >= 2")
    ap.add_argument("--fp32-check", type=int, default=1,
                    help="after the headline (bf16): the same size as an fp32 sum, exact-checked and timed (BASELINE.md "
                         "target 3 names both dtypes); 0 = skip")
    ap.add_argument("--sweep", default="auto",
                    help="after the headline timing: exact-checked size sweep MIN:MAX:FACTOR (nccl-tests style, "
                         "BASELINE.md target 3, peak busBW reported); 'auto' = 8:16G:8 on GPUs, 8:1M:8 for "
                         "--backend cpu; or 'off'")
    ap.add_argument("--ring-probe", default="auto", choices=["auto", "on", "off"],
                    help="K6 concurrent ring probe of the chosen subset (child process of rank 0, before any rank "
                         "touches its GPU): the busBW ceiling 'busbw_vs_probe_bound' divides by; auto = on at k >= 2 "
                         "when the link probe ran")
    ap.add_argument("--cpu-bind", default="auto", choices=["auto", "env", "off"],
                    help="Gaia B6: pin each rank to GTK_CPUSET (a pod's Allocate env) narrowed to its own device's core "
                         "slice, or to that slice on a bare node (auto); env = GTK_CPUSET only; off")
    ap.add_argument("--budget-s", type=float, default=300.0,
                    help="wall-clock budget: a supplementary phase (tuning, sweep, fp32, graph, worst-subset A/B) is "
                         "skipped when its predicted cost would overrun it; the headline is never skipped; 0 = no limit")
    ap.add_argument("--watchdog-s", type=float, default=None,
                    help="a rank still running after this many seconds (default: budget + 300; 0 = off) reports the "
                         "phase it is stuck in (rank 0: a JSON line, value null before the headline is timed and the measured "
                         "headline after it), dumps every thread's stack and "
                         "exits 124, so a hung collective ends the run with a diagnosis instead of a silent kill")
    return ap.parse_args(argv)


class Phases:
    """Per-phase wall time (``phase_s`` in the JSON line) and the ``--budget-s`` gate.  Decisions to
    skip a phase are agreed by every rank (MIN all-reduce), so no rank enters a collective alone."""

    def __init__(self, budget_s: float):
        self.t0 = time.perf_counter()
        self.budget = float(budget_s)
        self.s = {}
        self.skipped = []
        self.current = "setup"  # the phase in progress (the watchdog's report)
        self.headline = None  # the measured headline line, once timed (a later hang keeps it)

    def elapsed(self) -> float:
        return time.perf_counter() - self.t0

    def run(self, name, fn, *a, **kw):
        t = time.perf_counter()
        prev, self.current = self.current, name
        try:
            return fn(*a, **kw)
        finally:
            self.current = prev
            self.s[name] = round(self.s.get(name, 0.0) + time.perf_counter() - t, 3)

    def allow(self, name: str, predicted_s: float, agree=None) -> bool:
        ok = self.budget <= 0 or self.elapsed() + max(0.0, predicted_s) <= self.budget
        if agree is not None:
            ok = agree(ok)
        if not ok:
            self.skipped.append({"phase": name, "predicted_s": round(predicted_s, 2), "elapsed_s": round(self.elapsed(), 2)})
        return ok

    def report(self) -> dict:
        return dict(self.s, total=round(self.elapsed(), 3))


def start_watchdog(seconds: float, ph: Phases, rank: int, world: int, args, exit_fn=os._exit, out=None, err=None):
    """Arm a timer that ends a hung run with a diagnosis: the phase in progress (rank 0 prints the
    bench's JSON line with ``value: null`` and an ``error``), every thread's stack, exit code 124.
    A collective that never completes cannot be interrupted from Python, so the process exits
    (``os._exit``) instead of unwinding.  Returns the timer (``cancel()`` it once the line is out) or
    None when ``seconds <= 0``."""
    import faulthandler
    import threading

    if seconds is None or seconds <= 0:
        return None

    def fire():
        o = out or sys.stdout
        e = err or sys.stderr
        msg = f"watchdog: rank {rank} still in phase '{ph.current}' after {ph.elapsed():.0f} s"
        if rank == 0:
            if ph.headline is not None:
                # the headline was timed (max over ranks) before a supplementary phase hung: report it
                line = dict(ph.headline, error=msg + " (after the headline was measured)", phase_s=ph.report(),
                            skipped_phases=ph.skipped)
            else:
                line = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                        "warmup": args.warmup, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                        "dtype": args.dtype, "error": msg, "phase_s": ph.report()}
            print(json.dumps(line), file=o, flush=True)
        print(f"bench: {msg}; thread stacks follow", file=e, flush=True)
        try:
            faulthandler.dump_traceback(file=e, all_threads=True)
        except (AttributeError, ValueError, OSError):  # a stream without a file descriptor
            pass
        exit_fn(124)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def parse_size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(s[-1:], 1)
    return int(float(s[:-1] if mult > 1 else s) * mult)


def sweep_sizes(spec: str, cpu: bool = False):
    if spec == "off":
        return []
    if spec == "auto":
        spec = "8:1M:8" if cpu else "8:16G:8"
    lo, hi, fac = spec.split(":")
    lo, hi, fac = parse_size(lo), parse_size(hi), max(2, int(fac))
    out, b = [], lo
    while b <= hi:
        out.append(b)
        b *= fac
    if out and out[-1] < hi:
        out.append(hi)
    return out


def run_sweep(runner, sizes, env, tdev, barrier_kw, gpu_sync):
    """Every size: exact check, 1 warmup, then enough timed all-reduces for ~>=20 ms (max over
    ranks).  Returns nccl-tests style rows plus the peak busBW (algBW at k = 1)."""
    import torch
    import torch.distributed as dist

    from gpu_topology_on_k8s_amd.parallel.allreduce import bus_factor

    rows = []
    for b in sizes:
        runner.resize(b)
        wrong = torch.tensor([runner.check()], dtype=torch.int64, device=tdev)
        dist.all_reduce(wrong)
        runner.step()
        runner.synchronize()
        iters = 20 if b < (64 << 20) else (5 if b < (1 << 30) else 2)
        dist.barrier(**barrier_kw)
        gpu_sync()
        t0 = time.perf_counter()
        for _ in range(iters):
            runner.step()
        runner.synchronize()
        gpu_sync()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        us = float(t.item()) / iters * 1e6
        alg = runner.nbytes / (us * 1e-6) / 1e9
        rows.append({"bytes": runner.nbytes, "time_us": round(us, 2), "algbw_gbps": round(alg, 3),
                     "busbw_gbps": round(alg * bus_factor(env.world), 3), "wrong": int(wrong.item())})
    key = "busbw_gbps" if env.world > 1 else "algbw_gbps"
    peak = max(rows, key=lambda r: r[key]) if rows else None
    return {"rows": rows, "peak": {"bytes": peak["bytes"], key: peak[key]} if peak else None,
            "all_exact": all(r["wrong"] == 0 for r in rows)}


def run_other_dtype(runner, nbytes, dtype, env, tdev, barrier_kw, gpu_sync, steps):
    """BASELINE.md target 3 names bf16 AND fp32 sums: the same communicator re-prepared for ``dtype``
    at the headline size, exact-checked, then ``steps`` timed all-reduces (max over ranks)."""
    import torch
    import torch.distributed as dist

    from gpu_topology_on_k8s_amd.parallel.allreduce import bus_factor

    prev = runner.dtype
    runner.dtype = dtype
    try:
        runner.resize(nbytes)
        wrong = torch.tensor([runner.check()], dtype=torch.int64, device=tdev)
        dist.all_reduce(wrong)
        runner.step()
        runner.synchronize()
        dist.barrier(**barrier_kw)
        gpu_sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            runner.step()
        runner.synchronize()
        gpu_sync()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    finally:
        runner.dtype = prev
    ms = float(t.item()) / steps * 1e3
    alg = runner.nbytes / (ms / 1e3) / 1e9
    return {"dtype": dtype, "bytes": runner.nbytes, "steps": steps, "ms_per_step": round(ms, 4),
            "algbw_gbps": round(alg, 3), "busbw_gbps": round(alg * bus_factor(env.world), 3), "exact": int(wrong.item()) == 0}


def run_graph_latency(runner, sizes, env, tdev, barrier_kw, gpu_sync, ops: int = 32, replays: int = 8):
    """Launch-bound small messages: ``ops`` out-of-place all-reduces captured into one hipGraph
    (native ``Comm.capture``) and replayed, against the same ``ops`` enqueued one call at a time.
    µs per all-reduce, max over ranks; the graph's result is exact-checked (``Comm.verify``)."""
    import torch
    import torch.distributed as dist

    def timed(fn, n):
        dist.barrier(**barrier_kw)
        gpu_sync()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        runner.synchronize()
        gpu_sync()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    rows = []
    c = runner.comm
    for b in sizes:
        runner.resize(b)
        eager_us = timed(runner.step, ops * replays) / (ops * replays) * 1e6
        c.capture(ops, False)
        c.replay()
        runner.synchronize()
        graph_us = timed(c.replay, replays) / (ops * replays) * 1e6
        wrong = torch.tensor([c.verify()], dtype=torch.int64, device=tdev)
        dist.all_reduce(wrong)
        rows.append({"bytes": runner.nbytes, "eager_us": round(eager_us, 2), "graph_us": round(graph_us, 2),
                     "speedup": round(eager_us / graph_us, 2) if graph_us > 0 else None, "wrong": int(wrong.item())})
    return {"ops_per_graph": ops, "rows": rows, "all_exact": all(r["wrong"] == 0 for r in rows)}


def parse_ctas(spec: str):
    if spec in ("auto", "tune", "default"):
        return None
    lo, _, hi = spec.partition(":")
    return (int(lo), int(hi or 0))


def tune_ctas(env, device, nbytes, args, tdev, barrier_kw):
    """Untimed pass: one communicator per TUNE_CANDIDATES entry, ``--tune-steps`` all-reduces of the
    full message each (max over ranks); returns the fastest (min, max) and the table.  Every rank
    builds every candidate (init is collective) and agrees on the winner through an all-reduce."""
    import torch
    import torch.distributed as dist

    from gpu_topology_on_k8s_amd.parallel.allreduce import AllReduceRunner

    table = []
    best, best_ms = None, float("inf")
    for i, cand in enumerate(TUNE_CANDIDATES):
        try:
            r = AllReduceRunner(env, device, nbytes, args.dtype, backend="native", inplace=args.inplace,
                                ctas=cand if cand != (0, 0) else None, tag=f"/tune{i}")
            ok = 1
        except Exception as e:  # noqa: BLE001 - skipped by every rank together
            print(f"bench: ctas {cand} unavailable on rank {env.rank}: {e}", file=sys.stderr)
            r, ok = None, 0
        flag = torch.tensor([ok], dtype=torch.int32, device=tdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            if r is not None:
                r.close()
            continue
        r.step()
        r.synchronize()
        dist.barrier(**barrier_kw)
        t0 = time.perf_counter()
        for _ in range(max(1, args.tune_steps)):
            r.step()
        r.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item()) / max(1, args.tune_steps) * 1e3
        r.close()
        table.append({"ctas": list(cand), "ms_per_step": round(ms, 4)})
        if ms < best_ms:
            best, best_ms = cand, ms
    if best is None or best == (0, 0):
        return None, table
    return best, table


def measure_worst(env, choice, nbytes, args, tdev, barrier_kw, backend, ctas):
    """The placement A/B inside the north-star run: the worst-scoring k-subset of the same node."""
    return measure_subset(env, "worst", choice.worst, choice.worst_hip, choice.worst_score, nbytes, args, tdev, barrier_kw,
                          backend, ctas)


def measure_subset(env, label, subset, hip, score, nbytes, args, tdev, barrier_kw, backend, ctas):
    """One placement A/B arm: rank r builds a second communicator on ``hip[r]`` (another k-subset of the
    same node: the worst one, or the kubelet's default choice), checks it exactly and times
    ``min(K, 20)`` all-reduces of the headline size (max over ranks)."""
    import torch
    import torch.distributed as dist

    from gpu_topology_on_k8s_amd.parallel.allreduce import AllReduceRunner, bus_factor

    wdev = int((hip or subset)[env.rank])
    ok, r = 1, None
    try:
        r = AllReduceRunner(env, wdev, nbytes, args.dtype, backend=backend, inplace=args.inplace, ctas=ctas, tag=f"/{label}")
    except Exception as e:  # noqa: BLE001 - every rank learns it through the flag below
        print(f"bench: {label}-subset communicator unavailable on rank {env.rank}: {e}", file=sys.stderr)
        ok = 0
    flag = torch.tensor([ok], dtype=torch.int32, device=tdev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        if r is not None:
            r.close()
        return {"subset": subset, "error": "communicator unavailable"}
    try:
        wrong = torch.tensor([r.check()], dtype=torch.int64, device=tdev)
        dist.all_reduce(wrong)
        for _ in range(max(1, args.warmup // 2)):
            r.step()
        r.synchronize()
        steps = max(1, min(args.steps, 20))
        dist.barrier(**barrier_kw)
        t0 = time.perf_counter()
        for _ in range(steps):
            r.step()
        r.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item()) / steps * 1e3
        alg = r.nbytes / (ms / 1e3) / 1e9
        return {"subset": subset, "hip_devices": hip, "score": score, "steps": steps,
                "ms_per_step": round(ms, 4), "algbw_gbps": round(alg, 3), "busbw_gbps": round(alg * bus_factor(env.world), 3),
                "exact": int(wrong.item()) == 0}
    finally:
        r.close()


def _gain(ours: float, arm, world: int):
    """Headline rate over an A/B arm's (busBW at k >= 2, algBW at k = 1)."""
    key = "busbw_gbps" if world > 1 else "algbw_gbps"
    return round(ours / arm[key], 4) if arm and arm.get(key) else None


def _sweep_cost(sizes, algbw_gbps: float) -> float:
    """Predicted seconds of :func:`run_sweep` from the headline algBW (its iteration counts, plus a
    per-size overhead for the exact check and the warm-up op)."""
    bw = max(algbw_gbps, 1e-3) * 1e9
    t = 0.0
    for b in sizes:
        iters = 20 if b < (64 << 20) else (5 if b < (1 << 30) else 2)
        t += (iters + 2) * b / bw + 0.05
    return t


def main(argv=None) -> int:
    args = parse(argv)
    in_launcher = "WORLD_SIZE" in os.environ and "RANK" in os.environ
    if args.gpus > 1 and not in_launcher:
        # Re-launch under torch.distributed.run as a CHILD process (no exec; GPU untouched here).
        port = _free_port()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + (argv if argv is not None else sys.argv[1:])
        return subprocess.call(cmd)
    if not in_launcher:
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    # Cross-process GPU memory sharing (RCCL's P2P/IPC transport between the ranks' processes, k >= 2):
    # the amdgpu host driver of these nodes exports IPC handles only as dma-bufs, and the ROCr runtime
    # uses them only with the legacy KFD IPC path off; with it on, hipIpcGetMemHandle fails with
    # "invalid argument" and RCCL cannot open its peers' buffers.  Set before HIP initialises.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    ph = Phases(args.budget_s)
    wd_s = args.watchdog_s if args.watchdog_s is not None else (args.budget_s + 300.0 if args.budget_s > 0 else 0.0)
    watchdog = start_watchdog(wd_s, ph, int(os.environ.get("RANK", "0")), args.gpus, args)
    rccl_log = None
    if args.backend != "cpu" and (args.rccl_log == "on" or (args.rccl_log == "auto" and args.gpus > 1)) \
            and "NCCL_DEBUG" not in os.environ:
        from gpu_topology_on_k8s_amd.parallel.allreduce import rccl_log_env

        rccl_log = f"/tmp/gtk_rccl_{os.environ.get('MASTER_PORT', '0')}_{os.environ.get('RANK', '0')}"
        os.environ.update(rccl_log_env(rccl_log))  # before any communicator exists

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gpu_topology_on_k8s_amd.parallel.allreduce import (AllReduceRunner, DistEnv, SubsetChoice, bus_factor, choose_subset,
                                                             probe_node)
    from gpu_topology_on_k8s_amd.topology.cpus import bind_workload

    env = DistEnv.from_env()
    if env.world != args.gpus:
        print(f"bench: WORLD_SIZE={env.world} but --gpus={args.gpus}", file=sys.stderr)
        return 2
    cpu = args.backend == "cpu"
    dist.init_process_group(backend="gloo" if cpu else "nccl")
    env.store = dist.distributed_c10d._get_default_store()

    # --- placement: rank 0 picks the subset, everybody binds to subset[rank] ---------------------
    ring = None
    if env.rank == 0:
        preset = {"auto": None if cpu else "quick", "off": None}.get(args.probe, args.probe)
        topo = None
        if args.topology_json:
            from gpu_topology_on_k8s_amd.topology.model import Topology

            with open(args.topology_json) as f:
                topo = Topology.from_json(f.read())
            preset = None
        if preset:
            # the probe seeds the placement's cost matrix (scheduler-chosen subset): part of the
            # headline's definition, so it is bounded by the budget but never skipped
            tmo = 150.0 if args.budget_s <= 0 else max(30.0, min(150.0, args.budget_s / 3))
            topo, msg = ph.run("probe", probe_node, preset, backend=args.discovery, timeout=tmo)
            if topo is None:
                print(f"bench: link probe unavailable ({msg}); placing on discovered link classes", file=sys.stderr)
            elif msg != "ok":
                print(f"bench: link probe: {msg}", file=sys.stderr)
        choice = ph.run("place", choose_subset, env.world, backend=args.discovery,
                        visible=(args.cpu_visible or env.world) if cpu else None, topology=topo, via_k8s=args.via == "k8s")
        want_ring = args.ring_probe == "on" or (args.ring_probe == "auto" and env.world > 1 and choice.probed)
        if want_ring and not cpu and ph.allow("ring", 15.0):
            from gpu_topology_on_k8s_amd.ops.probe import ring_in_child

            # before any rank opens its GPU: the K6 child has the subset's links to itself
            ring, msg = ph.run("ring", ring_in_child, choice.hip_devices, preset or "quick")
            if ring is None:
                print(f"bench: ring probe unavailable ({msg})", file=sys.stderr)
                ring = {"error": msg[-300:]}
        env.store.set("gtk/subset", choice.to_json())
    choice = SubsetChoice.from_json(env.store.get("gtk/subset").decode())
    device = choice.hip_devices[env.rank]  # HIP ordinal of node device choice.devices[rank] (PCI-address map)
    tdev = "cpu" if cpu else f"cuda:{device}"
    barrier_kw = {} if cpu else {"device_ids": [device]}
    own = (choice.extra.get("cpusets") or [""] * env.world)[env.rank]
    cpu_rep = ph.run("cpu_bind", bind_workload, args.cpu_bind, own)
    env.store.set(f"gtk/cpuset/{env.rank}", json.dumps(cpu_rep))

    def gpu_sync():
        if not cpu:
            torch.cuda.synchronize()

    def agree(ok: bool) -> bool:
        f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=tdev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        return bool(int(f.item()))

    if not cpu:
        torch.cuda.set_device(device)

    nbytes = int(args.size_mb * (1 << 20))
    ctas = parse_ctas(args.ctas)
    tuning = None
    if args.backend == "native" and (args.ctas == "tune" or (args.ctas == "auto" and env.world > 1)):
        pred = len(TUNE_CANDIDATES) * (3.0 + (args.tune_steps + 1) * nbytes / 50e9)
        if ph.allow("tune", pred, agree):
            ctas, tuning = ph.run("tune", tune_ctas, env, device, nbytes, args, tdev, barrier_kw)
    runner = None
    t_comm = time.perf_counter()
    ph.current = "comm"
    if args.backend == "native":
        # The native communicator (csrc/rccl) is the measured path; if its extension cannot be
        # loaded on some rank, every rank falls back together to dist.all_reduce (the same RCCL).
        try:
            runner = AllReduceRunner(env, device, nbytes, args.dtype, backend="native", inplace=args.inplace,
                                     ctas=ctas, tag="/final")
            ok = 1
        except Exception as e:  # noqa: BLE001 - reported, then the whole job falls back
            print(f"bench: native RCCL communicator unavailable on rank {env.rank}: {e}", file=sys.stderr)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=tdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            if runner is not None:
                runner.close()
            runner = None
            args.backend = "torch"
    if runner is None:
        runner = AllReduceRunner(env, device, nbytes, args.dtype, backend=args.backend, inplace=args.inplace)
    comm_s = time.perf_counter() - t_comm
    ph.s["comm"] = round(comm_s, 3)
    ph.current = "setup"
    wrong = torch.tensor([ph.run("check", runner.check)], dtype=torch.int64, device=tdev)
    dist.all_reduce(wrong)
    if int(wrong.item()) != 0:
        print(f"bench: all-reduce correctness check FAILED ({int(wrong.item())} wrong elements)", file=sys.stderr)
        return 3

    def warm():
        for _ in range(args.warmup):
            runner.step()
        runner.synchronize()

    ph.run("warmup", warm)

    def headline():
        dist.barrier(**barrier_kw)
        gpu_sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            runner.step()
        runner.synchronize()
        gpu_sync()
        el = time.perf_counter() - t0
        dist.barrier(**barrier_kw)
        return el

    elapsed = ph.run("headline", headline)
    t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / max(1, args.steps) * 1e3
    algbw = runner.nbytes / (ms_per_step / 1e3) / 1e9  # headline size (the sweep below resizes)
    busbw = algbw * bus_factor(env.world)
    # whole-job aggregate (the bench contract): every rank's busBW summed, i.e. k x the per-rank
    # nccl-tests busBW (busbw_gbps below); at k = 1 busBW is 0 and the one rank's algBW is the value
    value = busbw * env.world if env.world > 1 else algbw
    headline_bytes = runner.nbytes
    ph.headline = {
        "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": env.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (rank-dependent exact pattern, verified before timing)",
        "config": {"model": "rccl-allreduce", "op": "sum", "message_bytes_per_gpu": headline_bytes, "inplace": args.inplace,
                   "backend": args.backend, "global_batch": None, "seq_len": None, "parallelism": f"dp{env.world}",
                   "subset": choice.devices, "hip_devices": choice.hip_devices},
        "algbw_gbps": round(algbw, 3), "busbw_gbps": round(busbw, 3), "scaling_comparable": env.world > 1,
    }
    step_s = ms_per_step / 1e3
    sweep = None
    sizes = sweep_sizes(args.sweep, cpu=cpu)
    if sizes and ph.allow("sweep", _sweep_cost(sizes, algbw), agree):
        try:  # supplementary: a failure here (e.g. no memory for 2 x 16 GiB) must not cost the headline
            sweep = ph.run("sweep", run_sweep, runner, sizes, env, tdev, barrier_kw, gpu_sync)
        except Exception as e:  # noqa: BLE001 - every rank runs the same sizes, so all land here together
            print(f"bench: size sweep aborted on rank {env.rank}: {e}", file=sys.stderr)
            sweep = {"error": str(e)[:300]}
    other = None
    fp32_steps = max(1, min(args.steps, 20))
    if args.fp32_check and runner.comm is not None and args.dtype != "fp32" \
            and ph.allow("fp32", (fp32_steps + 2) * step_s + 1.0, agree):
        try:  # supplementary, like the sweep
            other = ph.run("fp32", run_other_dtype, runner, headline_bytes, "fp32", env, tdev, barrier_kw, gpu_sync, fp32_steps)
        except Exception as e:  # noqa: BLE001
            print(f"bench: fp32 all-reduce aborted on rank {env.rank}: {e}", file=sys.stderr)
            other = {"dtype": "fp32", "error": str(e)[:300]}
    graph = None
    want_graph = args.graph == "on" or (args.graph == "auto" and env.world == 1)
    if want_graph and sizes and runner.comm is not None and not args.inplace and ph.allow("graph", 3.0, agree):
        try:  # supplementary, like the sweep
            graph = ph.run("graph", run_graph_latency, runner, [8, 4096, 65536, 1 << 20], env, tdev, barrier_kw, gpu_sync)
        except Exception as e:  # noqa: BLE001
            print(f"bench: graph latency aborted on rank {env.rank}: {e}", file=sys.stderr)
            graph = {"error": str(e)[:300]}
    worst_ab = None
    want_ab = args.ab_worst == "on" or (args.ab_worst == "auto" and bool(choice.worst))
    # a second communicator on other devices: the native RCCL comm (takes its device) or gloo on the CPU;
    # the torch backend's process group is bound to this rank's device
    if want_ab and choice.worst and (cpu or (choice.worst_hip and runner.comm is not None)) \
            and ph.allow("ab_worst", comm_s + (max(1, args.warmup // 2) + min(args.steps, 20) + 1) * step_s, agree):
        try:  # supplementary, like the sweep: a failure is reported, never costs the headline
            worst_ab = ph.run("ab_worst", measure_worst, env, choice, headline_bytes, args, tdev, barrier_kw, args.backend, ctas)
        except Exception as e:  # noqa: BLE001 - every rank runs the same steps
            print(f"bench: worst-subset A/B aborted on rank {env.rank}: {e}", file=sys.stderr)
            worst_ab = {"subset": choice.worst, "error": str(e)[:300]}
        finally:
            if not cpu:
                torch.cuda.set_device(device)  # the second communicator switched this thread's device
    default_ab = None
    want_default = args.ab_default == "on" or (args.ab_default == "auto" and bool(choice.default))
    if want_default and choice.default and worst_ab and not worst_ab.get("error") and sorted(choice.default) == sorted(choice.worst or []):
        default_ab = dict(worst_ab, same_as="worst")  # the kubelet's choice is the worst subset: measured once
    elif want_default and choice.default and (cpu or (choice.default_hip and runner.comm is not None)) \
            and ph.allow("ab_default", comm_s + (max(1, args.warmup // 2) + min(args.steps, 20) + 1) * step_s, agree):
        try:  # supplementary, like the worst-subset arm
            default_ab = ph.run("ab_default", measure_subset, env, "default", choice.default, choice.default_hip,
                                choice.default_score, headline_bytes, args, tdev, barrier_kw, args.backend, ctas)
        except Exception as e:  # noqa: BLE001
            print(f"bench: default-subset A/B aborted on rank {env.rank}: {e}", file=sys.stderr)
            default_ab = {"subset": choice.default, "error": str(e)[:300]}
        finally:
            if not cpu:
                torch.cuda.set_device(device)
    runner.close()
    rccl = None
    if rccl_log and env.rank == 0:
        from gpu_topology_on_k8s_amd.parallel.allreduce import rccl_log_summary

        path = f"{rccl_log}.{os.getpid()}"
        try:
            with open(path) as f:
                rccl = rccl_log_summary(f.read())
            rccl["log"] = path
        except Exception as e:  # noqa: BLE001 - supplementary: never costs the headline line
            rccl = {"error": str(e)[:200]}
    if env.rank == 0:
        probe = choice.extra.get("probe") or {}
        ingress = probe.get("subset_ingress_bound_gbps")  # K5/K1: one GPU's ingress, others idle
        ring_bound = (ring or {}).get("ring_bound_gbps")  # K6: every member loaded at once
        bound = ring_bound or ingress
        binds = []
        for r in range(env.world):
            try:
                binds.append(json.loads(env.store.get(f"gtk/cpuset/{r}").decode()))
            except Exception as e:  # noqa: BLE001 - reported, never costs the line
                binds.append({"applied": False, "reason": str(e)[:100]})
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": env.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (rank-dependent exact pattern, verified before timing)",
            "config": {
                "model": "rccl-allreduce",
                "op": "sum",
                "message_bytes_per_gpu": headline_bytes,
                "inplace": args.inplace,
                "backend": args.backend,
                "global_batch": None,
                "seq_len": None,
                "parallelism": f"dp{env.world}",
                "subset": choice.devices,
                "hip_devices": choice.hip_devices,
                "placement_score": choice.score,
                "placement_ms": choice.placement_ms,
                "worst_subset": choice.worst,
                "worst_score": choice.worst_score,
                "default_subset": choice.default,
                "default_score": choice.default_score,
                "topology_source": choice.source,
                "probed": choice.probed,
                "rccl_ctas": list(ctas) if ctas else "rccl-default",
            },
            "phase_s": ph.report(),
            "skipped_phases": ph.skipped,
            "budget_s": args.budget_s,
            "cpuset_applied": [{k: b.get(k) for k in ("applied", "source", "cpus", "n", "reason")} for b in binds],
            "ctas_tuning": tuning,
            "link_probe": choice.extra.get("probe"),
            "ring_probe": ring,
            "k8s_placement": choice.extra.get("k8s"),
            "size_sweep": sweep,
            "fp32_headline": other,
            "graph_latency": graph,
            "rccl": rccl,
            "worst_subset_ab": worst_ab,
            "placement_gain": _gain(busbw if env.world > 1 else algbw, worst_ab, env.world),
            "default_subset_ab": default_ab,
            "placement_gain_vs_default": _gain(busbw if env.world > 1 else algbw, default_ab, env.world),
            # the objective's terms of the chosen, worst and default subsets, what separates them and the
            # gain the slowest link predicts (placement/explain.py): a healthy xGMI mesh predicts 1.00
            "placement_terms": choice.extra.get("placement_terms"),
            "value_kind": ("aggregate busbw (k x per-rank busbw_gbps)" if env.world > 1
                           else "algbw (busbw = 0 at k=1)"),
            "busbw_vs_probe_bound": round(busbw / bound, 4) if bound else None,
            "probe_bound_kind": "k6-ring" if ring_bound else ("k5-ingress" if ingress else None),
            "algbw_gbps": round(algbw, 3),
            "busbw_gbps": round(busbw, 3),
            # k >= 2 values are aggregate busBW (k x the per-rank nccl-tests busBW); k = 1 has no bus
            # traffic (busBW = 0) and reports one rank's algBW, an HBM copy rate.  The two are different
            # quantities: nothing should divide one by the other
            "aggregate_busbw_gbps": round(busbw * env.world, 3) if env.world > 1 else None,
            "per_rank_busbw_gbps": round(busbw, 3) if env.world > 1 else None,
            "scaling_comparable": env.world > 1,
            "scaling_note": ("comparable across k >= 2 only: aggregate busBW over xGMI" if env.world > 1 else
                             "k=1: algBW of one rank's all-reduce = the HIP runtime's HBM device copy, not a bus rate; "
                             "not comparable to the k>=2 aggregate busBW values"),
        }
        if watchdog is not None:
            watchdog.cancel()
        print(json.dumps(out), flush=True)
    if watchdog is not None:
        watchdog.cancel()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
