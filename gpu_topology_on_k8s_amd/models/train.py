"""Data-parallel training on the scheduler-chosen devices: Llama-3 (BASELINE config 5) and the Gaia
paper's MNIST CNN (Exp. 6, ``models/mnist.py``).

    python -m torch.distributed.run --nproc-per-node K --master-addr 127.0.0.1 \
        -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 2 --seq 4096 --steps 10 --placement best
    ... -m gpu_topology_on_k8s_amd.models.train --model mnist-cnn --batch 64 --steps 200   # images/s, epoch time

One process per GPU; rank 0 discovers the node, runs the placement core for the k-subset (``best``)
or its worst-scoring alternative (``worst``), and every rank binds to ``subset[rank]`` — what the pod
would see after the device plugin's Allocate.  A step = forward + backward with bucketed RCCL
gradient all-reduce overlapped with backward + global-norm clip + fused AdamW.  Reports tokens/s
(whole job) and model FLOP utilisation against the 2.5 PF/s dense bf16 peak per GPU.
Runs on CPU with the gloo backend for tests (tiny model).

``--graph on`` captures the whole step (device-side batch synthesis, forward, backward, gradient
all-reduce, clipping, capturable AdamW) into one hipGraph after the warmup and replays it: the mode
for launch-bound models such as the MNIST CNN ('auto' = on for MNIST at world 1 on a GPU).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

from .llama import Llama, LlamaConfig
from .mnist import EPOCH_IMAGES, MnistCNN, MnistConfig
from .gemm_tuning import setup_gemm_tuning
from .optim import FlatAdamW, FlatSGD
from .checkpoint import CheckpointWriter, load_checkpoint
from ..parallel.dp import DEFAULT_COMM_CTAS, BucketedAllReduce, broadcast_params
from ..topology.cpus import bind_workload

__all__ = ["train", "main"]

PEAK_BF16_FLOPS = 2.5e15  # MI355X dense bf16 (MI355X_MICROARCH.md), per GPU


AUTO_CTAS = (32, 64, 128)  # --comm-ctas auto: the candidates around the one-GPU shadow sweep's knee


def _comm_group(ctas: int):
    """A process group over every rank with RCCL's CTAs per collective capped at ``ctas`` (gloo: a
    plain group, so the selection logic runs in CPU tests)."""
    if dist.get_backend() == "nccl":
        from ..parallel.dp import nccl_options

        return dist.new_group(backend="nccl", pg_options=nccl_options(max_ctas=ctas))
    return dist.new_group(backend="gloo")


def _init_dist(device_kind: str, comm_ctas=0) -> Dict[str, int]:
    if "RANK" not in os.environ:
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if not dist.is_initialized():
        # rehearsal (GTK_REHEARSE_ON_ONE_GPU=1): every rank on the one visible GPU, collectives over
        # gloo (RCCL refuses two ranks on one device) — the multi-rank DP / ZeRO-1 GPU code paths run
        # on a single-GPU box; production runs one rank per GPU over RCCL
        rehearse = device_kind == "cuda" and os.environ.get("GTK_REHEARSE_ON_ONE_GPU") == "1"
        backend = "gloo" if rehearse or device_kind != "cuda" else "nccl"
        kw = {}
        if backend == "nccl" and comm_ctas and comm_ctas != "auto":
            from ..parallel.dp import nccl_options

            kw["pg_options"] = nccl_options(max_ctas=comm_ctas)  # RCCL's CTAs per collective, capped
        dist.init_process_group(backend=backend, **kw)
    return {"rank": rank, "world": world, "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}


def _pod_devices(env, visible_bdfs=None) -> Dict[str, object]:
    """Inside a pod: train on the devices the device plugin allocated (``GTK_GPU_GROUP`` node-local
    indices, ``GTK_GPU_BDFS`` their PCI addresses; ``design.md:239``), rank r on GROUP[r], mapped to
    this container's HIP ordinals by PCI address (:func:`topology.identity.resolve_group`)."""
    from ..topology.identity import ENV_GROUP, fractions_from_env, group_from_env, resolve_group

    group, bdfs = group_from_env()
    if len(group) != env["world"]:
        raise ValueError(f"{ENV_GROUP}={group} allocates {len(group)} devices for a job of {env['world']} ranks")
    hip = resolve_group(group, bdfs=bdfs or None, visible_bdfs=visible_bdfs)
    fr = fractions_from_env()
    return {"devices": group, "hip_devices": hip, "best": group, "best_score": None, "worst": None, "worst_score": None,
            "source": "pod-allocation", "fractions": fr if len(fr) == len(group) else None}


def apply_share_cap(pl: Dict[str, object], rank: int, dev: int) -> Optional[float]:
    """On a time-sliced node (``GTK_GPU_FRACTION``, topology/shares.py) hold this process to its
    share of the GPU's HBM: the caching allocator refuses to grow past ``fraction * capacity``.  The
    compute side of the share is the slices' disjoint CUs (``HSA_CU_MASK`` from Allocate, with the
    plugin's ``--share-cu-mask on``); HBM is shared by the slices, so this cap is the cooperative
    part of the share.  Returns the cap."""
    fr = pl.get("fractions")
    if not fr or float(fr[rank]) >= 1.0:
        return None
    if os.environ.get("GTK_VGPU_ACTIVE") == "1":
        # the vGPU guard (libgtk_vgpu.so, preloaded by Allocate) already enforces the share and reports
        # it as the device's total through hipMemGetInfo, which is what the allocator's memory
        # fraction is taken of: capping again would leave fraction x share
        return float(fr[rank])
    torch.cuda.set_per_process_memory_fraction(float(fr[rank]), dev)
    return float(fr[rank])


def _choose_device(env, placement: str, discovery: str, visible: Optional[int] = None) -> Dict[str, object]:
    """Rank 0 places the job; the choice travels through the store.  ``visible`` models a node of
    that many devices without HIP (CPU dry runs of the best-vs-worst harness on a fake node)."""
    store = dist.distributed_c10d._get_default_store()
    if env["rank"] == 0:
        from ..parallel.allreduce import choose_subset

        topo = None
        if os.environ.get("GTK_TOPOLOGY_JSON"):  # a node model to place on (CPU rehearsals of the A/B)
            from ..topology.model import Topology

            with open(os.environ["GTK_TOPOLOGY_JSON"]) as f:
                topo = Topology.from_json(f.read())
        ch = choose_subset(env["world"], backend=discovery, visible=visible, topology=topo)
        # best = the placement core; worst = its highest-objective alternative; default = what the
        # kubelet hands out with no extender (the paper's default-Kubernetes comparator): the best set
        # again when the kubelet would pick the same devices
        arm = {"worst": (ch.worst, ch.worst_hip, "worst_cpusets"),
               "default": (ch.default, ch.default_hip, "default_cpusets")}.get(placement)
        use = arm if arm and arm[0] else None
        devices = use[0] if use else ch.devices  # node-local topology indices (GROUP numbering)
        info = {"devices": devices, "hip_devices": use[1] if use else ch.hip_devices, "best": ch.devices,
                "best_score": ch.score, "worst": ch.worst, "worst_score": ch.worst_score, "default": ch.default,
                "default_score": ch.default_score, "source": ch.source,
                "placement_terms": ch.extra.get("placement_terms"),
                # Gaia B6: each rank's share of the node's cores, the slice of its own device
                "cpusets": ch.extra.get(use[2]) if use else ch.extra.get("cpusets")}
        store.set("gtk/train_placement", json.dumps(info))
    return json.loads(store.get("gtk/train_placement").decode())


def train(model_name: str = "tiny", batch: int = 1, seq: int = 128, steps: int = 3, warmup: int = 1, device_kind: str = "cuda",
          placement: str = "auto", discovery: str = "auto", bucket_mb: float = 256.0, checkpoint: bool = False, lr: float = 3e-4,
          attn: str = "hip", seed: int = 0, log: bool = True, gemm_tuning: str = "auto",
          gemm_table: Optional[str] = None, gemm_layout: str = "nt",
          zero1: bool = False, save_dir: Optional[str] = None, save_every: int = 0, resume: Optional[str] = None,
          keep: int = 2, same_data: bool = False,
          graph: str = "auto", conv: str = "hip", cpu_bind: str = "auto", repeat_batch: bool = False,
          persistent_wt: bool = True, grad_reduce: str = "bf16", comm_ctas="auto",
          comm_shadow: int = 0, comm_shadow_k: int = 8, comm_shadow_busbw: float = 350.0,
          optimizer: str = "adamw", check_reduction: bool = False, data_ranks: int = 0, dropout: bool = True,
          fingerprint: bool = False) -> Dict[str, object]:
    """``optimizer="sgd"``, ``data_ranks``, ``fingerprint`` and ``check_reduction`` are the data-parallel
    correctness checks; see :func:`main`'s help for each."""
    if optimizer not in ("adamw", "sgd"):
        raise ValueError("optimizer must be 'adamw' or 'sgd'")
    if optimizer == "sgd" and (save_dir or resume):
        raise ValueError("--optimizer sgd is a parity check: it is not checkpointed")
    env = _init_dist(device_kind, comm_ctas)
    if placement == "auto":  # inside a pod the allocation decides; on a bare node, the placement core
        placement = "pod" if os.environ.get("GTK_GPU_GROUP") else "best"
    if device_kind == "cuda" and placement == "pod":
        pl = _pod_devices(env)
        dev = int(pl["hip_devices"][env["rank"]])
        torch.cuda.set_device(dev)
        pl["hbm_cap_fraction"] = apply_share_cap(pl, env["rank"], dev)
        device = torch.device("cuda", dev)
        gemm_mode = setup_gemm_tuning(gemm_tuning, gemm_table, env["rank"])
    elif device_kind == "cuda" and os.environ.get("GTK_REHEARSE_ON_ONE_GPU") == "1":
        pl = {"devices": [0] * env["world"], "hip_devices": [0] * env["world"], "best": [0], "worst": None, "source": "rehearsal"}
        torch.cuda.set_device(0)
        device = torch.device("cuda", 0)
        gemm_mode = setup_gemm_tuning(gemm_tuning, gemm_table, env["rank"])
    elif device_kind == "cuda":
        pl = _choose_device(env, placement, discovery)
        dev = int(pl["hip_devices"][env["rank"]])
        torch.cuda.set_device(dev)
        device = torch.device("cuda", dev)
        gemm_mode = setup_gemm_tuning(gemm_tuning, gemm_table, env["rank"])
    else:
        if discovery == "fake":  # placement on a fake node (GTK_FAKE_GPUS devices), ranks stay on the CPU
            pl = _choose_device(env, placement, discovery, visible=int(os.environ.get("GTK_FAKE_GPUS", "8")))
        else:
            pl = {"devices": [], "best": [], "worst": None, "source": "cpu"}
        device = torch.device("cpu")
        gemm_mode = "off"
    # Gaia B6 (paper p.3 "GPU and CPU core are automatically bound"): pin this rank to GTK_CPUSET (the
    # pod's Allocate env) narrowed to its own device's core slice, or to that slice on a bare node,
    # before the model, the optimizer and the data path start their host threads
    own = ""
    cs = pl.get("cpusets")
    if cs and env["rank"] < len(cs):
        own = cs[env["rank"]] or ""
    cpu_rep = bind_workload(cpu_bind if device_kind == "cuda" else ("env" if cpu_bind == "auto" else cpu_bind), own)
    mnist = model_name.startswith("mnist")
    use_graph = graph == "on" or (graph == "auto" and mnist and device.type == "cuda" and env["world"] == 1)
    if use_graph and device.type != "cuda":
        raise ValueError("--graph on needs a GPU")
    if use_graph and zero1:
        raise ValueError("--graph does not capture ZeRO-1's per-bucket weight all-gathers")
    # data: rank r draws from seed 1234 + r (1234 for every rank with --same-data); --data-ranks K makes
    # ONE rank draw every one of K ranks' batches and train on their concatenation -- the batch a K-rank
    # job's gradient all-reduce averages over, for the k-rank vs 1-rank parity check
    if data_ranks and env["world"] != 1:
        raise ValueError("--data-ranks emulates K ranks' data on a 1-rank job")
    seeds = [1234 + i for i in range(data_ranks)] if data_ranks else [1234 + (0 if same_data else env["rank"])]
    data_seed = seeds[0]
    local_batch = batch * len(seeds)
    if mnist:
        cfg = MnistConfig.named(model_name)
        if not dropout:  # deterministic in the batch split: what the k-rank vs 1-rank parity check needs
            cfg = dataclasses.replace(cfg, p1=0.0, p2=0.0)
        model = MnistCNN(cfg, device=device, seed=seed, conv=conv)
        items_per_step, unit, flops_per_item = local_batch, "images", cfg.flops_per_image()
    else:
        cfg = LlamaConfig.named(model_name)
        model = Llama(cfg, device=device, seed=seed, checkpoint=checkpoint, attn=attn, gemm_layout=gemm_layout,
                      persistent_wt=persistent_wt)
        items_per_step, unit, flops_per_item = local_batch * seq, "tokens", cfg.flops_per_token(seq)
    broadcast_params(model.flat)
    # graph mode issues the gradient collectives after backward (inside the captured step), not from
    # autograd hooks mid-backward: one capture-friendly sequence
    shadow = None
    if comm_shadow and env["world"] == 1 and device.type == "cuda":
        # what a k-GPU DP step's collectives take from this GPU: CTA-limited paced copies from the
        # bucket hooks (parallel/dp.py CommShadow, profiles/r04_comm_shadow)
        from ..parallel.dp import CommShadow

        shadow = CommShadow(device, comm_shadow, k=comm_shadow_k, busbw_gbps=comm_shadow_busbw,
                            max_bucket_bytes=int(bucket_mb * (1 << 20)))
    def make_ar(group=None) -> BucketedAllReduce:
        return BucketedAllReduce(model.flat, group=group, bucket_mb=bucket_mb, zero1=zero1, overlap=not use_graph,
                                 grad_reduce=grad_reduce, shadow=shadow)

    ar = make_ar()
    if optimizer == "sgd":
        if use_graph and getattr(model.flat, "data_t", None) is not None:
            raise ValueError("--optimizer sgd with --graph: the captured step would keep a stale W^T")
        opt = FlatSGD(model.flat, lr=lr, shards=ar.shards() if zero1 else None, capturable=use_graph)
    else:
        opt = FlatAdamW(model.flat, lr=lr, shards=ar.shards() if zero1 else None, capturable=use_graph)
    if zero1:
        model.param_ready = ar.wait_param
    if mnist and use_graph:
        model.step_counter = opt.t_dev  # dropout hash keyed by the device step count (advances per replay)
    # same_data: every rank draws rank 0's batches, so the averaged gradient equals the 1-rank
    # gradient and a k-rank run must reproduce the 1-rank losses (the DP correctness check).
    # MNIST batches are synthesised on the device; in graph mode by the mnist_synth kernel, indexed
    # by the optimizer's device step counter (dropout masks from the graph-safe default generator).
    if mnist and use_graph:
        torch.cuda.manual_seed(data_seed)
        gen = None
        gens = []
    else:
        gens = [torch.Generator(device=device if mnist else "cpu").manual_seed(sd) for sd in seeds]
        gen = gens[0]
    def update_fp():
        """Four fixed pseudo-random projections (fp64) of the fp32 master weights: every rank sums its
        1/world partition of each bucket and the sums are all-reduced, so a k-rank job and a 1-rank job
        produce comparable numbers.  Their change over a run fingerprints the weight update."""
        acc = torch.zeros(4, dtype=torch.float64, device=opt.master.device)
        base, o = {}, 0
        for s_, e_ in opt.shards:  # flat offset -> offset in the optimizer's (concatenated) master
            base[(s_, e_)] = o
            o += e_ - s_
        for b in ar.buckets:
            lo = b.start + (b.numel * env["rank"]) // env["world"]
            hi = b.start + (b.numel * (env["rank"] + 1)) // env["world"]
            for (s_, e_), o_ in base.items():
                a0, a1 = max(lo, s_), min(hi, e_)
                for a in range(a0, a1, 1 << 24):
                    z = min(a1, a + (1 << 24))
                    w = opt.master[o_ + a - s_:o_ + z - s_].double()
                    idx = torch.arange(a, z, dtype=torch.float64, device=w.device)
                    for k in range(4):
                        acc[k] += (w * torch.sin(idx * (0.6180339887 + 0.1 * k) + k)).sum()
        if env["world"] > 1:
            dist.all_reduce(acc)
        return acc.tolist()

    fp0 = update_fp() if fingerprint else None
    start_step, resumed = 0, None
    if resume:
        meta = load_checkpoint(resume, model, opt, gen)
        start_step, resumed = int(meta["step"]), meta["path"]
    ckpt = CheckpointWriter(save_dir, model, opt, model_name=model_name, keep=keep, zero1=zero1) if save_dir else None
    if ckpt is not None and save_every > 0:
        ckpt.prepare()
    done = [start_step]
    first: Dict[str, object] = {}

    def _cat(parts):
        return parts[0] if len(parts) == 1 else tuple(torch.cat(z) for z in zip(*parts))

    def batch_tokens():
        if mnist and use_graph:  # one HIP launch per seed, indexed by the optimizer's device step counter
            x, y = _cat([model.synthetic_batch_dev(batch, opt.t_dev, seed=sd) for sd in seeds])
            return x.contiguous(memory_format=torch.channels_last), y
        if mnist:
            x, y = _cat([model.synthetic_batch(batch, g) for g in gens])
            return x.contiguous(memory_format=torch.channels_last), y
        if repeat_batch and "t" in first:  # memorisation check: the same tokens every step
            t = first["t"]
        else:
            t = torch.cat([torch.randint(0, cfg.vocab, (batch, seq + 1), generator=g) for g in gens])
            t = first["t"] = t.to(device, non_blocking=True)
        return t[:, :-1], t[:, 1:]

    def body(xy=None, before_opt=None) -> torch.Tensor:
        x, y = xy if xy is not None else batch_tokens()
        model.flat.zero_grad()
        loss = model(x, y)
        loss.backward()
        ar.finish()
        if before_opt is not None:
            before_opt()
        opt.step(grad_scale=ar.grad_scale, grad=ar.reduced_grad)
        ar.gather_params()  # zero1: overlaps the next forward; no-op otherwise
        return loss.detach()

    # --check-reduction: the first step checks the gradient reduction with DIFFERENT data per rank.  A
    # hook-free pass of the same batch (same dropout state) gives each rank's local gradient; the real
    # pass then copies every bucket's input right before its collective launches.  Checked, on the
    # stream and at the point the optimizer reads it: the reduced buffer against the fp64 sum of all
    # ranks' local gradients (a skipped bucket, an unawaited collective, a wrong scale fail), and each
    # launched bucket against the local gradient (a bucket whose collective started before backward
    # finished writing it fails).  In graph mode the copies are captured with the step and the check
    # runs after the first replay (a replay that re-ran a stale collective fails).
    check = {"pending": bool(check_reduction), "result": None}
    tol = 1e-3 if ar.grad32 is not None else 1e-2

    def _rng():
        st = {"cpu": torch.get_rng_state()}
        if device.type == "cuda":
            st["cuda"] = torch.cuda.get_rng_state(device)
        if getattr(model, "_own_step", None) is not None:
            st["own"] = model._own_step.clone()
        return st

    def _set_rng(st):
        torch.set_rng_state(st["cpu"])
        if "cuda" in st:
            torch.cuda.set_rng_state(st["cuda"], device)
        if "own" in st:
            model._own_step.copy_(st["own"])

    def _record(red, rdy) -> None:
        ok = red["max_rel"] <= tol and (rdy is None or rdy["max_rel"] <= tol)
        check["result"] = {"ok": bool(ok), "tol": tol, "reduce_max_rel": red["max_rel"],
                           "ready_max_rel": None if rdy is None else rdy["max_rel"], "buckets": len(red["buckets"]),
                           "worst_bucket": max(red["buckets"], key=lambda z: z["rel"])["index"] if red["buckets"] else None,
                           "mode": "graph-replay" if use_graph else "eager", "world": env["world"]}

    def checked_body() -> torch.Tensor:
        xy = batch_tokens()
        st = _rng()
        ar.suspend(True)
        model.flat.zero_grad()
        model(*xy).backward()
        if hasattr(model.flat, "fill_unwritten"):
            model.flat.fill_unwritten()
        ar.suspend(False)
        local = model.flat.grad.clone()
        _set_rng(st)
        ar.capture_local(True)

        def verify():
            frozen = ar.freeze()  # what the optimizer reads, before the check's own collectives run
            ar.capture_local(False)
            _record(ar.verify(local, frozen=frozen), ar.verify(local, against=ar.snapshot) if env["world"] > 1 else None)

        return body(xy, before_opt=verify)

    captured = {}

    def capture() -> None:
        """After the eager warmup (library handles, workspaces and autotuning exist): record one
        whole step into a hipGraph; it is not executed here."""
        torch.cuda.synchronize(device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            captured["loss"] = body()
        captured["g"] = g
        torch.cuda.synchronize(device)

    def step() -> torch.Tensor:
        if "g" in captured:
            captured["g"].replay()
            opt.note_replay()
            loss = captured["loss"].clone()
            if check["pending"]:
                check["pending"] = False
                _record(ar.verify(ar.snapshot if env["world"] > 1 else ar.reduced_buffer()), None)
        elif check["pending"] and not use_graph:
            check["pending"] = False
            loss = checked_body()
        else:
            loss = body()
        done[0] += 1
        if ckpt is not None and save_every > 0 and done[0] % save_every == 0:
            ar.wait_all_params()
            ckpt.save(done[0], gen)
        return loss

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    losses = []
    for _ in range(max(warmup, 1) if use_graph else warmup):
        losses.append(step())
    ar.wait_all_params()
    cta_table = None
    if comm_ctas == "auto" and env["world"] > 1 and not use_graph:
        # the first k >= 2 run confirms the CTA cap the one-GPU comm shadow chose:
        # one communicator per candidate cap; on each a settling pass and two timed passes (max over
        # ranks) of forward + backward with the bucketed reductions overlapped (+ ZeRO-1's all-gather
        # of the unchanged weights) -- no optimizer update, one fixed batch, the data generators and
        # dropout state restored after -- so training is exactly the run without the tuning.
        cta_table, groups = [], {}
        gstates = [g.get_state() for g in gens]
        rng0 = _rng()
        first0 = dict(first)
        xy = batch_tokens()

        def tune_pass():
            model.flat.zero_grad()
            model(*xy).backward()
            ar.finish()
            ar.gather_params()
            ar.wait_all_params()

        for c in AUTO_CTAS:
            groups[c] = _comm_group(c)
            ar.remove()
            ar = make_ar(groups[c])
            if zero1:
                model.param_ready = ar.wait_param
            tune_pass()
            sync()
            dist.barrier()
            ta = time.perf_counter()
            for _ in range(2):
                tune_pass()
            sync()
            tt = torch.tensor([time.perf_counter() - ta], dtype=torch.float64,
                              device=device if device.type == "cuda" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            cta_table.append({"ctas": c, "ms_per_pass": float(tt.item()) / 2 * 1e3})
        best = min(cta_table, key=lambda r: r["ms_per_pass"])["ctas"]
        ar.remove()
        ar = make_ar(groups[best])
        for c, grp in groups.items():  # the losers' communicators (RCCL: channel buffers per peer) go now
            if c != best:
                dist.destroy_process_group(grp)
        if zero1:
            model.param_ready = ar.wait_param
        comm_ctas = best
        for g, st_ in zip(gens, gstates):
            g.set_state(st_)
        _set_rng(rng0)
        first.clear()
        first.update(first0)
    if use_graph:
        if check["pending"]:
            ar.capture_local(True)  # the captured finish() copies every bucket's input before its collective
        capture()
    sync()
    dist.barrier()
    sync()
    if shadow is not None:
        shadow.reset_timing()
    t0 = time.perf_counter()
    for _ in range(steps):
        losses.append(step())
    ar.wait_all_params()
    sync()
    dt = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([dt], dtype=torch.float64, device=device if device.type == "cuda" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    fp1 = update_fp() if fingerprint else None
    if ckpt is not None:
        if not ckpt.has(done[0]):
            ckpt.save(done[0], gen)
        ckpt.close()
    items = env["world"] * items_per_step * steps
    tps = items / dt
    mfu = tps * flops_per_item / (PEAK_BF16_FLOPS * env["world"]) if device.type == "cuda" else None
    out = {
        "metric": (f"{'MNIST CNN' if mnist else 'Llama'} DP training {unit}/s on the scheduler-chosen subset"),
        "model": model_name,
        "throughput": tps,
        "throughput_unit": f"{unit}/s",
        "graph": use_graph,
        "conv": getattr(model, "conv", None),
        "params": cfg.num_params(),
        "n_gpus": env["world"],
        "placement": placement,
        "devices": pl["devices"],
        "placement_source": pl.get("source"),
        "gpu_fractions": pl.get("fractions"),
        "hbm_cap_fraction": pl.get("hbm_cap_fraction"),
        "best_devices": pl.get("best"),
        "worst_devices": pl.get("worst"),
        "default_devices": pl.get("default"),
        "best_score": pl.get("best_score"),
        "worst_score": pl.get("worst_score"),
        "default_score": pl.get("default_score"),
        "placement_terms": pl.get("placement_terms"),
        "global_batch": local_batch * env["world"],
        "seq_len": None if mnist else seq,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": dt / max(1, steps) * 1e3,
        "tokens_per_s": None if mnist else tps,
        "images_per_s": tps if mnist else None,
        "epoch_s": EPOCH_IMAGES / tps if mnist else None,  # one 60k-image MNIST epoch at the measured rate
        "mfu": mfu,
        "loss_first": float(losses[0]),
        "loss_last": float(losses[-1]),
        "losses": [float(x) for x in losses],
        "same_data": same_data,
        "data_ranks": data_ranks or None,
        "optimizer": optimizer,
        "dropout": dropout,
        "check_reduction": check["result"] if check_reduction else None,
        "update_fingerprint": [b - a for a, b in zip(fp0, fp1)] if fingerprint else None,
        "repeat_batch": repeat_batch,
        "lr": lr,
        "buckets": ar.stats["buckets"],
        "zero1": zero1,
        "optimizer_state_gb": opt.state_bytes() / 1e9,
        "bucket_mb": bucket_mb,
        "gemm_tuning": gemm_mode,
        "gemm_layout": gemm_layout,
        "grad_reduce": grad_reduce,
        "comm_ctas": comm_ctas or None,
        "comm_ctas_tuning": cta_table,
        "comm_shadow": ({"ctas": shadow.ctas, "k": shadow.k, "busbw_gbps": shadow.busbw,
                         "collectives_per_step": shadow.launched / max(1, done[0] - start_step),
                         "ring_bytes_per_step": shadow.bytes / max(1, done[0] - start_step),
                         "collective_us_per_step": shadow.micros / max(1, done[0] - start_step),
                         **shadow.timing()}
                        if shadow is not None else None),
        "persistent_wt": bool(getattr(model, "persistent_wt", False)),
        "attn_ot": getattr(model, "attn_ot", None),
        "flat_grads": bool(getattr(model, "flat_grads", False)),
        "optimizer_writes_wt": bool(getattr(opt, "fused_t", False)),
        "wt_refreshes": int(getattr(model.flat, "t_refreshes", 0)),
        "step_start": start_step,
        "step_end": done[0],
        "resumed_from": resumed,
        "checkpoints_saved": ckpt.saved if ckpt is not None else [],
        "checkpoint_stats": ckpt.stats if ckpt is not None else None,
        "max_mem_gb": (torch.cuda.max_memory_allocated(device) / 1e9) if device.type == "cuda" else None,
        "cpuset_applied": {k: cpu_rep.get(k) for k in ("applied", "source", "cpus", "n", "reason")},
        # a time-sliced share's container tier (libgtk_vgpu.so preloaded by Allocate) in force in this process
        "share_guard": os.environ.get("GTK_VGPU_ACTIVE") == "1",
    }
    if log and env["rank"] == 0:
        print(json.dumps(out), flush=True)
    ar.remove()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="llama3-8b", choices=["llama3-8b", "llama3-1b", "tiny", "mnist-cnn"])
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--placement", default="auto", choices=["auto", "best", "worst", "default", "pod"],
                    help="pod = the devices Allocate gave this container (GTK_GPU_GROUP/GTK_GPU_BDFS); best/worst = "
                         "run the placement core on the node; default = the devices the kubelet hands out with no "
                         "extender (lowest free indices); auto = pod when GTK_GPU_GROUP is set, else best")
    ap.add_argument("--discovery", default="auto")
    ap.add_argument("--bucket-mb", type=float, default=256.0)
    ap.add_argument("--checkpoint", action="store_true")
    ap.add_argument("--attn", default="hip", choices=["hip", "sdpa", "sdpa-expand"])
    ap.add_argument("--gemm-tuning", default="auto", choices=["auto", "off", "use", "tune"],
                    help="TunableOp library-GEMM selection (models/gemm_tuning.py)")
    ap.add_argument("--gemm-table", default=None, help="TunableOp results table (default: the shipped MI355X table)")
    ap.add_argument("--zero1", action="store_true",
                    help="shard the optimizer over the ranks: reduce-scatter grads, all-gather weights (ZeRO-1)")
    ap.add_argument("--save-dir", default=None, help="write checkpoints here (async; at the end, and every --save-every steps)")
    ap.add_argument("--save-every", type=int, default=0, help="checkpoint interval in optimizer steps (0 = only at the end)")
    ap.add_argument("--keep", type=int, default=2, help="committed checkpoints to keep")
    ap.add_argument("--resume", default=None,
                    help="checkpoint root (its latest) or step directory; any world size / --zero1 setting")
    ap.add_argument("--same-data", action="store_true",
                    help="every rank trains on rank 0's batches (k-rank losses must equal the 1-rank run)")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="capture the whole step into one hipGraph after warmup (auto: MNIST at world 1 on a GPU)")
    ap.add_argument("--conv", default="hip", choices=["hip", "torch"],
                    help="MNIST convolution stack: hip = csrc/ops/mnist_conv.hip (MFMA), torch = MIOpen via F.conv2d")
    ap.add_argument("--cpu-bind", default="auto", choices=["auto", "env", "off"],
                    help="Gaia B6: pin this rank to GTK_CPUSET narrowed to its device's core slice (auto; on a bare node the "
                         "slice alone), GTK_CPUSET only (env), or leave the threads unbound (off)")
    ap.add_argument("--repeat-batch", action="store_true",
                    help="train on the first batch at every step: uniform random tokens carry nothing to learn, one "
                         "repeated batch does, so the loss must fall (end-to-end check of forward, backward and AdamW)")
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--optimizer", default="adamw", choices=["adamw", "sgd"],
                    help="sgd: plain SGD on the fp32 master (the DP parity check: unlike AdamW, its update is linear "
                         "in the gradient, so a reduction that did not run changes it)")
    ap.add_argument("--check-reduction", action="store_true",
                    help="check the first step's gradient reduction with different data per rank: the buffer the "
                         "optimizer reads against the fp64 sum of every rank's local gradient (bf16 <= 1e-2, fp32 <= "
                         "1e-3 relative, per bucket) and each bucket's collective input against the complete local "
                         "gradient; the job exits 3 when it fails")
    ap.add_argument("--data-ranks", type=int, default=0,
                    help="1-rank job: train on the concatenation of these many ranks' batches (the k-rank parity "
                         "reference)")
    ap.add_argument("--dropout", default="on", choices=["on", "off"],
                    help="MNIST dropout (off: the forward does not depend on how the batch is split over ranks)")
    ap.add_argument("--fingerprint", action="store_true",
                    help="report update_fingerprint: fixed projections of the fp32 master weights' change over the run")
    ap.add_argument("--grad-reduce", default="bf16", choices=["bf16", "fp32"],
                    help="DP gradient reduction dtype: bf16 in place, or fp32 (a widened copy reduced and applied in fp32)")
    ap.add_argument("--comm-ctas", default="auto", type=lambda v: v if v == "auto" else int(v),
                    help="cap RCCL's CTAs per collective (ncclConfig_t maxCTAs; 0 = RCCL's choice; N = that cap); "
                         f"auto (world > 1): time {'/'.join(map(str, AUTO_CTAS))} after the warmup and keep the fastest "
                         f"(reported as comm_ctas_tuning); at world 1 nothing to cap.  {DEFAULT_COMM_CTAS} is the knee of "
                         "the one-GPU comm-shadow sweep (profiles/r04_comm_shadow)")
    ap.add_argument("--comm-shadow", type=int, default=0,
                    help="one GPU: play each bucket's k-GPU ring all-reduce as this many CU-holding workgroups (0 = off)")
    ap.add_argument("--comm-shadow-k", type=int, default=8, help="--comm-shadow: ranks of the emulated ring")
    ap.add_argument("--comm-shadow-busbw", type=float, default=350.0,
                    help="--comm-shadow: per-rank bus GB/s that sets each emulated collective's duration")
    a = ap.parse_args(argv)
    out = train(a.model, a.batch, a.seq, a.steps, a.warmup, a.device, a.placement, a.discovery, a.bucket_mb, a.checkpoint, lr=a.lr, attn=a.attn,
          gemm_tuning=a.gemm_tuning, gemm_table=a.gemm_table, zero1=a.zero1, save_dir=a.save_dir, save_every=a.save_every,
          resume=a.resume, keep=a.keep, same_data=a.same_data, graph=a.graph, conv=a.conv, cpu_bind=a.cpu_bind,
          repeat_batch=a.repeat_batch, grad_reduce=a.grad_reduce, comm_ctas=a.comm_ctas, comm_shadow=a.comm_shadow,
          comm_shadow_k=a.comm_shadow_k, comm_shadow_busbw=a.comm_shadow_busbw, optimizer=a.optimizer,
          check_reduction=a.check_reduction, data_ranks=a.data_ranks, dropout=a.dropout == "on", fingerprint=a.fingerprint)
    if dist.is_initialized():
        dist.destroy_process_group()
    cr = out.get("check_reduction")
    if a.check_reduction and not (cr and cr.get("ok")):
        print(json.dumps({"check_reduction_failed": cr}), file=sys.stderr, flush=True)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
