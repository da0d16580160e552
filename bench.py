#!/usr/bin/env python
"""Benchmark of the differential-attention hot path on MI355X.

Default (``--mode kernel``): BASELINE.json configs[1] -- the fused N=2
differential-attention core, bf16, B=8 per GPU, H=16, head_size=64, dv=128,
T=4096, causal, forward + backward, on synthetic N(0,1) inputs resident in HBM.
One step = one forward + one backward of that core over one batch.  With N
GPUs (torchrun, one process per GPU over RCCL) every rank runs its own batch
shard: the path shards by batch with no data-path collective ("weak" scaling);
only the timing uses a barrier and a MAX all-reduce.

``value`` = algorithmic TFLOP/s of the whole job: ranks x 3*F_fwd per step /
step time, F_fwd = B*H*T^2*(N*hs + dv) (causal-halved matmul FLOPs).
``roofline`` reports the dominant kernel (the fused backward) from HIP events
bracketing its launches inside the timed region.  ``cpu_baseline`` times the CPU
oracle (the reference's algorithm op for op: per-head loop, materialised T x T
maps, fp32) on a bounded sample on this host.

The kernel line also carries:
  ``train``        BASELINE configs[3] -- the ~350M DiffTransformer DP training
                   step (bucketed RCCL all-reduce overlapped with backward) at
                   this run's world size: whole-job train tokens/s, so the 1/2/4/8
                   GPU lines give the train scaling curve (``--train-steps 0`` skips);
  ``hbm_kernels``  the HBM-bound norm / RoPE kernels at their BASELINE shapes
                   (GroupLayerNorm fwd/bwd at cfg2's 32768 x 2048, RoPE at cfg3),
                   HIP-event times and GB/s against 8 TB/s.

``--mode train``: data-parallel training tokens/s of a reference-architecture
model (see differential_transformer_replication_amd/train.py).

Launch: ``torchrun --nproc-per-node N ... bench.py --gpus N`` (one rank per GPU,
RCCL), or plain ``python bench.py --gpus N``, which spawns the N ranks itself
before anything touches the GPU.  ``--device cpu`` is a CPU/gloo dry run of the
multi-rank path (train leg only, a small control model).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "diff-attn fwd+bwd TFLOP/s (% MFMA peak); train tokens/sec at 1/2/4/8 GPUs"
PEAK_BF16_TFLOPS = 2516.6          # 256 CU x 2.4 GHz x 4096 flop/clk/CU (dense, MI355X_MICROARCH.md)


def _dist(device="cuda"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device == "cpu":
        if world > 1:
            dist.init_process_group("gloo")
        return world, rank, local
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def _sync(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()


def _max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], device="cuda", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _host_threads() -> int:
    """Host threads this process may use: OMP_NUM_THREADS when the launcher sets it
    (the GPU box sets its CPU share, 16, there), else the CPUs in our affinity mask
    (os.cpu_count() reports the whole machine on the box)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(T=4096, H=16, hs=64, reps=2):
    """Oracle (reference algorithm, eager fp32, per-head loop) on the host CPU.
    Bounded sample: B=1, H=16 at the full T; heads and batch entries are
    independent so the rate per FLOP carries to B=8.  Inputs are drawn before the
    timed region; the oracle keeps the reference's persistent causal mask
    (a ``tril`` built once, compared per call: diff_transformer.py:31,61-62)."""
    from oracle import diffattn_oracle as orc
    threads = _host_threads()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    dv = 2 * hs
    heads = []
    for _h in range(H):
        q = [torch.randn(1, T, hs, generator=g, requires_grad=True) for _ in range(2)]
        k = [torch.randn(1, T, hs, generator=g, requires_grad=True) for _ in range(2)]
        v = torch.randn(1, T, dv, generator=g, requires_grad=True)
        heads.append((q, k, v, torch.randn(1, T, dv, generator=g)))
    lam = torch.tensor(0.47, requires_grad=True)
    orc.causal_softmax(heads[0][0][0][:, :8].detach(), heads[0][1][0][:, :8].detach(), 0.125)   # warm
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for q, k, v, do in heads:
            coef = torch.stack([torch.ones(()), -lam])
            out = orc.diff_core(q, k, v, coef)
            out.backward(do)
        ts.append(time.perf_counter() - t0)
    f_fwd, f_bwd = orc.flops_attention(1, H, T, hs, dv, 2)
    sec = sum(ts) / len(ts)
    return {"value": round((f_fwd + f_bwd) / sec / 1e12, 6), "unit": "TFLOP/s", "cores": threads,
            "kind": "port",
            "sample": f"CPU oracle (reference algorithm op for op, eager fp32, per-head loop, materialised "
                      f"T x T maps) fwd+bwd of B=1 H={H} T={T} hs={hs} N=2, mean of {reps}; "
                      f"{sec:.2f} s per sample; rate per algorithmic FLOP, same FLOP count as the GPU step; "
                      f"fidelity vs the reference itself: profiles/r02_cpu_fidelity.json"}


DEFAULT_SHAPE = "B8_H16_hs64_N2_T4096_dv128"       # cfg2, the default kernel workload


def shape_key(B, H, hs, N, T, dv) -> str:
    return f"B{B}_H{H}_hs{hs}_N{N}_T{T}_dv{dv}"


def lib_sha() -> str:
    """First 16 hex digits of sha256(libdiffattn.so): the kernel build being run."""
    import hashlib
    path = os.path.join(ROOT, "differential_transformer_replication_amd", "lib", "libdiffattn.so")
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def _pmc_traffic(kernel, shape=DEFAULT_SHAPE):
    """HBM bytes per launch of ``kernel`` at workload ``shape`` from the newest
    committed PMC summary for that shape (profiles/*_pmc_traffic.json, written
    from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled
    per the gfx950 correction), and only one taken on the kernel build this run
    loads (its ``lib_sha``): counters of an older build are never paired with this
    build's timings.  Summaries without a "shape" field were all taken on the
    default cfg2 command.  (None, None) when no summary matches."""
    import glob
    import re
    cur = lib_sha()
    nat = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), key=nat)  # rNN_vM: newest last
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
            legacy = ("decode_" if kernel.startswith("decode") else "") + DEFAULT_SHAPE
            if d.get("shape", legacy) != shape or d.get("lib_sha") != cur:
                continue
            k = d["kernels"].get(kernel)
        except (OSError, ValueError, KeyError):
            continue
        if k:
            return k["traffic_bytes"], os.path.relpath(f, ROOT)
    return None, None


def _sq_clock(kernel, shape=DEFAULT_SHAPE):
    """Effective clock of ``kernel`` under load (GRBM_GUI_ACTIVE / 8 / dispatch duration,
    MI355X_MICROARCH.md 'DVFS give-back') from the newest committed SQ summary
    (profiles/*_sq.json, tools/pmc_sq.py) taken on this run's kernel build at this
    workload shape.  (None, None) when no summary matches."""
    import glob
    import re
    cur = lib_sha()
    nat = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))]
    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_sq.json")), key=nat)):
        try:
            with open(f) as fh:
                d = json.load(fh)
            if d.get("lib_sha") != cur or d.get("shape", DEFAULT_SHAPE) != shape:
                continue
            ghz = d["kernels"][kernel.replace("attn_bwd_", "attn_")]["clock_ghz"]
        except (OSError, ValueError, KeyError):
            continue
        return ghz, os.path.relpath(f, ROOT)
    return None, None


def control_bench(B, H, hs, T, steps, warmup):
    """control.py's standard causal attention (control.py:38-63) at equal F_fwd, on
    PyTorch's own fused GPU attention (SDPA), bf16 fwd+bwd: the comparison line of
    BASELINE configs[4].  Returns (ms per step, algorithmic TFLOP/s)."""
    import torch.nn.functional as F
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(7)
    q, k, v = (torch.randn(B, H, T, hs, device=dev, dtype=torch.bfloat16, generator=g).requires_grad_(True)
               for _ in range(3))
    do = torch.randn(B, H, T, hs, device=dev, dtype=torch.bfloat16, generator=g)

    def step():
        for t in (q, k, v):
            t.grad = None
        F.scaled_dot_product_attention(q, k, v, is_causal=True).backward(do)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / steps
    f = 3.0 * B * H * T * T * (hs + hs)          # N=1, dv=hs: F_fwd = B H T^2 (hs + dv)
    return sec * 1e3, f / sec / 1e12


def control_fused_bench(B, H, hs, T, steps, warmup):
    """The same control attention on this repo's fused kernels (N=1, coef 1, dv=hs):
    the like-for-like comparison of BASELINE configs[4].  Returns (ms, TFLOP/s)."""
    from differential_transformer_replication_amd import ops
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(7)
    W = ops.packed_width(H, 1, hs, hs)
    qkv = torch.randn(B, T, W, device=dev, dtype=torch.bfloat16, generator=g).requires_grad_(True)
    do = torch.randn(B, T, H * hs, device=dev, dtype=torch.bfloat16, generator=g)
    coef = torch.ones(H, 1, device=dev, dtype=torch.float32)

    def step():
        qkv.grad = None
        ops.diff_attention(qkv, coef, H, 1, hs, dv=hs).backward(do)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / steps
    f = 3.0 * B * H * T * T * (hs + hs)
    return sec * 1e3, f / sec / 1e12


def _coefficients(H, N, hs, dev):
    """Seeded branch coefficients: lambda_* ~ N(0, 0.1) at layer 3."""
    from differential_transformer_replication_amd.diff_transformer import _layer_lambda_coef
    from differential_transformer_replication_amd.Ndiff_transformer import alternating_coefficients
    from differential_transformer_replication_amd._compat import lambda_init_value
    g1 = torch.Generator(device=dev).manual_seed(1)
    if N == 1:
        return torch.ones(H, 1, device=dev)
    if N == 2:
        lam = [torch.randn(H, hs, device=dev, generator=g1) * 0.1 for _ in range(4)]
        return _layer_lambda_coef(*lam, lambda_init_value(3, None))
    lqs, lks = (torch.randn(H, N, hs, device=dev, generator=g1) * 0.1 for _ in range(2))   # Ndiff_transformer.py:79-93
    return alternating_coefficients(lqs, lks, float(lambda_init_value(3, None)))


def core_run(B, H, hs, N, T, steps, warmup, world=1, rank=0, dv=None):
    """Forward + backward of the fused attention core (bf16, causal, synthetic N(0,1)
    inputs resident in HBM) ``steps`` times after ``warmup``; the wall time of the
    timed region (barrier + synchronize on both sides, MAX over ranks) and every
    kernel's mean HIP-event time with its algorithmic TFLOP/s."""
    from differential_transformer_replication_amd import ops
    dv = 2 * hs if dv is None else dv
    dev = torch.device("cuda", torch.cuda.current_device())
    W = ops.packed_width(H, N, hs, dv)
    g = torch.Generator(device=dev).manual_seed(0 + rank)
    qkv = torch.randn(B, T, W, device=dev, dtype=torch.bfloat16, generator=g).requires_grad_(True)
    do = torch.randn(B, T, H * dv, device=dev, dtype=torch.bfloat16, generator=g)
    coef = _coefficients(H, N, hs, dev)

    def step():
        qkv.grad = None
        out = ops.diff_attention(qkv, coef, H, N, hs, dv=dv)
        out.backward(do)

    for _ in range(warmup):
        step()
    _sync(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _sync(world)
    el = time.perf_counter() - t0
    el = _max_over_ranks(el, world)
    # per-kernel HIP-event times from a second pass of the same steps, after the timed region:
    # the six events per step add gaps between the launches (tools/host_overhead_probe.py: cfg3
    # N = 3 1.066 -> 1.151 ms per step with them, cfg2 2.880 -> 2.904), so they stay out of it
    ops.TIMER.start()
    for _ in range(steps):
        step()
    ops.TIMER.stop()
    kt = ops.TIMER.mean_ms()
    f_fwd = float(B) * H * T * T * (N * hs + dv)
    f_bwd = 2 * f_fwd
    # per-kernel algorithmic FLOPs: the forward does F_fwd; the backward's 2*F_fwd is split by
    # its two kernels' products: dq (dQ = dS K) and dkdv (dV = P^T dO, dK = dS^T Q, dP = dO V^T)
    dq_share = N * hs / (2.0 * (N * hs + dv))
    flops = {"attn_fwd": f_fwd, "attn_bwd_dq": f_bwd * dq_share, "attn_bwd_dkdv": f_bwd * (1 - dq_share)}
    kernels = {}
    for name, (t, n) in kt.items():
        kernels[name] = {"ms": round(t, 4), "launches": n, "alg_tflops": round(flops[name] / t / 1e9, 2)}
    del qkv, do
    return el / steps, f_fwd + f_bwd, kernels


def kernel_bench(args, world, rank):
    B, H, hs, N, T = args.batch, args.heads, args.head_size, args.n_terms, args.seq
    dv = 2 * hs
    sec, flop, kernels = core_run(B, H, hs, N, T, args.steps, args.warmup, world, rank)
    ms = sec * 1e3
    value = world * flop / sec / 1e12
    dom = max(kernels, key=lambda k: kernels[k]["ms"])
    achieved = kernels[dom]["alg_tflops"]
    traffic, traffic_src = args.traffic, None
    if traffic is None:
        traffic, traffic_src = _pmc_traffic(dom, shape_key(B, H, hs, N, T, dv))
    ghz, ghz_src = _sq_clock(dom, shape_key(B, H, hs, N, T, dv))
    cfg2 = (B, H, hs, N, T) == (8, 16, 64, 2, 4096)
    workload = ("cfg2: fused N=2 diff-attention core fwd+bwd (BASELINE configs[1])" if cfg2 else
                f"diff-attention core fwd+bwd B={B} H={H} hs={hs} N={N} T={T}")
    res = {
        "metric": METRIC, "value": round(value, 3), "unit": "TFLOP/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": workload,
                   "batch_per_gpu": B, "global_batch": B * world, "heads": H, "head_size": hs, "dv": dv,
                   "seq_len": T, "n_terms": N, "causal": True,
                   "parallelism": f"batch-sharded replicas x{world} (no data-path collective)"},
        "mfma_frac_step": round(value / world / PEAK_BF16_TFLOPS, 4),
        "kernels": kernels,
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": achieved, "peak": PEAK_BF16_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     # the chip holds ~1.8-1.9 GHz under this load, not the 2.4 GHz the peak assumes:
                     # the MFMA peak at the measured clock, and the fraction of it
                     "clock_ghz": ghz, "clock_source": ghz_src,
                     "peak_at_clock": round(PEAK_BF16_TFLOPS * ghz / 2.4, 1) if ghz else None,
                     "frac_at_clock": round(achieved / (PEAK_BF16_TFLOPS * ghz / 2.4), 4) if ghz else None},
        "lib_sha": lib_sha(),
    }
    if args.control and rank == 0:
        # control.py standard attention at equal F_fwd: 2*H heads of width hs, dv = hs (train.py:226)
        Hc = 2 * H if N == 2 else H
        cms, ctf = control_bench(B, Hc, hs, T, args.steps, args.warmup)
        fms, ftf = control_fused_bench(B, Hc, hs, T, args.steps, args.warmup)
        res["control"] = {"what": "control.py causal softmax attention (control.py:38-63), bf16 fwd+bwd, "
                                  f"B={B} H={Hc} hs=dv={hs} T={T}",
                          "same_kernel": {"how": "this repo's fused kernels, N=1, coef 1, dv=hs (SURVEY 8f item 2)",
                                          "ms_per_step": round(fms, 4), "alg_tflops": round(ftf, 2),
                                          "diff_over_control_time": round(ms / fms, 3)},
                          "torch_sdpa": {"how": "torch scaled_dot_product_attention (ROCm fused attention)",
                                         "ms_per_step": round(cms, 4), "alg_tflops": round(ctf, 2),
                                         "diff_over_control_time": round(ms / cms, 3)}}
    return res


def configs_leg(args):
    """BASELINE configs[2] and [4] in the default line (one GPU, rank 0 only, short runs):
      cfg3  AlternatingDiffTransformer(12000, 768, 6, 10, 2048, n_terms=3 / 4) training step
            (bf16 autocast, micro-batch 16 x 2048): tokens/s and MFU, plus the attention
            core alone at that shape (B=16, H=6, hs=64, T=2048) with every kernel's
            algorithmic TFLOP/s;
      cfg5  the long-context core, B=1, H=16, hs=128 (dv=256), T=32768, N=2, against
            control.py's standard attention on the SAME kernels (N=1, coef 1, H=32,
            hs=dv=128: equal algorithmic FLOPs, train.py:226's n_head*2)."""
    out = {}
    for n in (3, 4):
        # each training leg in a fresh child process (the same command as a standalone
        # `bench.py --mode train --model ndiff` run): inside this process, after the other
        # legs, the N=3 step measured 65-79 ms against 51.5 ms standalone on the same box
        cmd = [sys.executable, os.path.abspath(__file__), "--mode", "train", "--model", "ndiff", "--n-terms", str(n),
               "--steps", str(args.cfg_steps), "--warmup", "3", "--cpu-baseline", "off"]
        proc = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if proc.returncode != 0:
            raise RuntimeError(f"cfg3 n_terms={n} leg failed: {proc.stderr[-2000:]}")
        r = json.loads(proc.stdout.strip().splitlines()[-1])
        torch.cuda.empty_cache()
        # warm after the training leg's idle host time: the step is ~1.1 ms, so 30 warm-up steps
        # (~35 ms) before 30 timed ones (a 10-step sample after 5 read 5-10% slow, r06l vs r06z probe)
        sec, flop, kernels = core_run(16, 6, 64, n, 2048, max(args.cfg_steps, 30), 30)
        out[f"cfg3_n{n}"] = {"train_tokens_per_s": r["value"], "train_ms_per_step": r["ms_per_step"],
                             "mfu": r.get("mfu"), "params": r["config"]["params"],
                             "core": {"shape": "B=16 H=6 hs=64 dv=128 T=2048 bf16 causal", "ms_per_step": round(
                                 sec * 1e3, 4), "alg_tflops": round(flop / sec / 1e12, 2), "kernels": kernels}}
    torch.cuda.empty_cache()
    sec, flop, kernels = core_run(1, 16, 128, 2, 32768, max(2, args.cfg_steps // 2), 1)
    torch.cuda.empty_cache()
    csec, cflop, ckernels = core_run(1, 32, 128, 1, 32768, max(2, args.cfg_steps // 2), 1, dv=128)
    out["cfg5"] = {"diff": {"shape": "B=1 H=16 hs=128 dv=256 N=2 T=32768 bf16 causal", "ms_per_step": round(sec * 1e3, 3),
                            "alg_tflops": round(flop / sec / 1e12, 2), "kernels": kernels},
                   "control_same_kernel": {"shape": "B=1 H=32 hs=dv=128 N=1 T=32768 bf16 causal (control.py:38-63)",
                                           "ms_per_step": round(csec * 1e3, 3),
                                           "alg_tflops": round(cflop / csec / 1e12, 2), "kernels": ckernels},
                   "diff_over_control_time": round(sec / csec, 3)}
    return out


def decode_bench(args, world, rank):
    """--mode decode: one KV-cache decode launch (dta_attn_decode) per step, bf16,
    cache length L = --seq.  HBM-bound: algorithmic bytes per launch =
    B*H*L*(N*hs + dv)*2 (every cached K_i / V row read once)."""
    from differential_transformer_replication_amd import ops
    B, H, hs, N, L = args.batch, args.heads, args.head_size, args.n_terms, args.seq
    dv = 2 * hs
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(0)
    k = torch.randn(B, L, H, N, hs, device=dev, dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, L, H, dv, device=dev, dtype=torch.bfloat16, generator=g)
    q = torch.randn(B, H, N, hs, device=dev, dtype=torch.bfloat16, generator=g)
    coef = torch.tensor([[1.0, -0.5, 0.3, -0.2][:N]] * H, device=dev)
    for _ in range(args.warmup):
        ops.diff_attention_decode(q, k, v, coef, L)
    _sync(world)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record()
        ops.diff_attention_decode(q, k, v, coef, L)
        e1.record()
    _sync(world)
    ms = _max_over_ranks((time.perf_counter() - t0) * 1e3 / args.steps, world)
    kms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    nbytes = B * H * L * (N * hs + dv) * 2
    return {"metric": "KV-cache decode attention GB/s (one new token per sequence)", "value": round(
        world * nbytes / ms / 1e6, 1), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16", "data": "synthetic",
        "config": {"workload": "decode: one query row per (b, h) over an L-row KV cache", "batch_per_gpu": B,
                   "heads": H, "head_size": hs, "dv": dv, "n_terms": N, "cache_len": L},
        "roofline": {"bound": "hbm", "kernel": "decode_kernel", "achieved": round(nbytes / kms / 1e6, 1),
                     "peak": 8000.0, "unit": "GB/s", "frac": round(nbytes / kms / 1e6 / 8000.0, 4),
                     "traffic": _decode_traffic(B, H, hs, N, L), "kernel_ms": round(kms, 5), "alg_bytes": nbytes}}


def _decode_traffic(B, H, hs, N, L):
    # PMC bytes of the split + combine launches, only for the default decode shape they were measured on
    if (B, H, hs, N, L) != (8, 16, 64, 2, 4096):
        return None
    parts = [_pmc_traffic(k, "decode_" + shape_key(B, H, hs, N, L, 2 * hs))[0] for k in ("decode_split", "decode_combine")]
    return None if None in parts else sum(parts)


def hbm_bench(reps=20):
    """The HBM-bound kernels around the attention core, at BASELINE shapes, timed
    with HIP events on the launch stream (median of ``reps``):
      ln_fwd / ln_bwd  GroupLayerNorm x0.2 (diff_transformer.py:15-20, 90-91) at cfg2:
                       B*T = 32768 rows x C' = H*dv = 2048, bf16;
                       algorithmic bytes fwd 2*rows*C'*2 (read x, write y),
                       bwd 3*rows*C'*2 (read x and dy, write dx);
      rope             interleaved-pair RoPE of every Q_i/K_i (Ndiff_transformer.py:11-22)
                       at cfg3: B=16, T=2048, 2H=12 (Q and K of H=6 heads), N=3, hs=64,
                       bf16; bytes 2 * elements * 2 (read, write; the fp32 table is
                       T*hs*4 and stays in cache)."""
    from differential_transformer_replication_amd import ops, _lib
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(3)
    out = {}
    rows, C = 8 * 4096, 16 * 128
    x = torch.randn(rows, C, device=dev, dtype=torch.bfloat16, generator=g)
    w = torch.ones(C, device=dev) + 0.1 * torch.randn(C, device=dev, generator=g)
    b = 0.1 * torch.randn(C, device=dev, generator=g)
    dy = torch.randn(rows, C, device=dev, dtype=torch.bfloat16, generator=g)

    def timed(fn):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(a.elapsed_time(b_) for a, b_ in ev)
        return ts[len(ts) // 2]

    lib = _lib.load()
    stream = _lib.stream_handle(dev)
    y = torch.empty_like(x)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    dx = torch.empty_like(x)
    dw = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    fa = _lib.LnArgs(_lib.DTA_BF16, rows, C, 1e-5, 0.2, x.data_ptr(), C, y.data_ptr(), C, w.data_ptr(),
                     b.data_ptr(), mean.data_ptr(), rstd.data_ptr(), None, 0, None, 0, None, None)
    part = torch.empty(lib.dta_ln_bwd_workspace_bytes(rows, C) // 4, device=dev)
    ba = _lib.LnArgs(_lib.DTA_BF16, rows, C, 1e-5, 0.2, x.data_ptr(), C, None, 0, w.data_ptr(), None,
                     mean.data_ptr(), rstd.data_ptr(), dy.data_ptr(), C, dx.data_ptr(), C, dw.data_ptr(),
                     db.data_ptr(), part.data_ptr())
    ms_f = timed(lambda: _lib.check(lib.dta_ln_fwd(fa, stream)))
    # the production backward: ln_bwd + the ordered reduce of its column partials (dw/db accumulate: values unused)
    ms_b = timed(lambda: _lib.check(lib.dta_ln_bwd(ba, stream)))
    for name, ms, nbytes in (("ln_fwd", ms_f, 2 * rows * C * 2), ("ln_bwd", ms_b, 3 * rows * C * 2)):
        out[name] = {"us": round(ms * 1e3, 2), "alg_bytes": nbytes, "GBps": round(nbytes / ms / 1e6, 1),
                     "frac_of_8TBps": round(nbytes / ms / 1e6 / 8000.0, 4)}
    B, T, H2, N, hs = 16, 2048, 12, 3, 64
    src = torch.randn(B, T, H2, N, hs, device=dev, dtype=torch.bfloat16, generator=g)
    dst = torch.empty_like(src)
    from differential_transformer_replication_amd.Ndiff_transformer import precompute_freqs_cis
    table = torch.view_as_real(precompute_freqs_cis(hs, T)).to(dev).contiguous()
    ms_r = timed(lambda: ops.rope_rows(src, dst, table))
    nbytes = 2 * src.numel() * 2
    out["rope"] = {"us": round(ms_r * 1e3, 2), "alg_bytes": nbytes, "GBps": round(nbytes / ms_r / 1e6, 1),
                   "frac_of_8TBps": round(nbytes / ms_r / 1e6 / 8000.0, 4),
                   "shape": f"B={B} T={T} 2H={H2} N={N} hs={hs} bf16"}
    del x, y, dy, dx, src, dst
    return out


def train_leg(args, world, rank):
    """BASELINE configs[3] DP training step (cfg4) at this run's world size.  At one GPU the
    step launches no collective; it then runs a second time over a 1-rank RCCL process group
    with every gradient bucket's all-reduce launched from the backward hooks
    (BucketedAllReduce(reduce_single=True)): the difference is the hook / launch / RCCL
    overhead an N-rank step carries on top of its xGMI transfer time."""
    from differential_transformer_replication_amd.train import train_bench
    targs = argparse.Namespace(steps=args.train_steps, warmup=args.train_warmup, model="diff",
                               n_terms=args.n_terms, device=args.device)
    r = train_bench(targs, world, rank)
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "final_loss", "config",
            "model_tflops", "mfu")
    out = {k: r[k] for k in keep if k in r}
    if world == 1 and args.device == "cuda" and args.rccl_world1:
        torch.cuda.empty_cache()
        own = not dist.is_initialized()
        # RCCL prints a version banner on stdout when the communicator comes up: keep this
        # process's stdout to the one JSON line (fd 1 -> fd 2 for the leg)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if own:
                import socket
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    port = sk.getsockname()[1]
                dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                        device_id=torch.device("cuda", torch.cuda.current_device()))
            r1 = train_bench(argparse.Namespace(**vars(targs), reduce_single=True), 1, 0)
            out["rccl_hooks_world1"] = {
                "what": "the same cfg4 step with every bucket all-reduce launched from the backward hooks over a "
                        "1-rank RCCL group (no xGMI traffic): hook + launch + RCCL overhead per step",
                "value": r1["value"], "ms_per_step": r1["ms_per_step"],
                "overhead_ms": round(r1["ms_per_step"] - r["ms_per_step"], 3),
                "parallelism": r1["config"]["parallelism"]}
        except Exception as e:          # report, never fail the bench line over the probe
            out["rccl_hooks_world1"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        finally:
            if own and dist.is_initialized():
                dist.destroy_process_group()
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return out


def run(args):
    world, rank, local = _dist(args.device)
    if args.device == "cpu":
        # CPU / gloo dry run of the multi-rank path: the train leg on a small control model
        from differential_transformer_replication_amd.train import train_bench
        targs = argparse.Namespace(steps=args.steps, warmup=args.warmup, model="cpu-dry", n_terms=args.n_terms,
                                   device="cpu")
        res = train_bench(targs, world, rank)
        res["cpu_baseline"] = None
    elif args.mode == "kernel":
        # the train leg first: run after the kernel and HBM legs in the same process it
        # measured 7-8% below a --mode train run on the same box
        train = None
        if args.train_steps > 0 and os.environ.get("DTA_TRAIN_LEG_FIRST", "1") != "0":
            train = train_leg(args, world, rank)
            torch.cuda.empty_cache()
        res = kernel_bench(args, world, rank)
        if rank == 0 and args.hbm:
            res["hbm_kernels"] = hbm_bench()
        if world == 1 and args.configs and args.cfg_steps > 0:
            torch.cuda.empty_cache()
            res["configs"] = configs_leg(args)
        if args.train_steps > 0:
            if train is None:
                torch.cuda.empty_cache()
                train = train_leg(args, world, rank)
            res["train"] = train
    elif args.mode == "decode":
        res = decode_bench(args, world, rank)
    else:
        from differential_transformer_replication_amd.train import train_bench
        res = train_bench(args, world, rank)
    if rank == 0:
        default_kernel = args.mode == "kernel" and args.device == "cuda" and (
            args.batch, args.heads, args.head_size, args.n_terms, args.seq) == (8, 16, 64, 2, 4096)
        if args.cpu_baseline == "auto" and world == 1 and default_kernel:
            res["cpu_baseline"] = cpu_baseline()
        elif "cpu_baseline" not in res:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _rank_main(rank, args, world, port):
    # a spawned rank: the same environment torchrun would give it
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    run(args)


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["kernel", "train", "decode"], default="kernel")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: gloo dry run of the multi-rank path (train leg on a small control model)")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--head-size", type=int, default=64)
    ap.add_argument("--n-terms", type=int, default=2)
    ap.add_argument("--control", action="store_true",
                    help="kernel mode: also time control.py standard attention at equal F_fwd (BASELINE configs[4])")
    ap.add_argument("--model", choices=["diff", "ndiff"], default="diff",
                    help="train mode: cfg4 DiffTransformer (diff) or cfg3 AlternatingDiffTransformer (ndiff)")
    ap.add_argument("--train-steps", type=int, default=8,
                    help="kernel mode: timed steps of the cfg4 DP training leg (0 = skip)")
    ap.add_argument("--train-warmup", type=int, default=3)
    ap.add_argument("--no-rccl-world1", dest="rccl_world1", action="store_false",
                    help="kernel mode, one GPU: skip the second cfg4 train leg over a 1-rank RCCL group")
    ap.add_argument("--no-hbm", dest="hbm", action="store_false", help="kernel mode: skip the LN / RoPE timings")
    ap.add_argument("--no-configs", dest="configs", action="store_false",
                    help="kernel mode: skip the cfg3 / cfg5 legs (one GPU only)")
    ap.add_argument("--cfg-steps", type=int, default=10, help="timed steps of each cfg3 / cfg5 leg")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per dominant-kernel launch from rocprofv3 PMC (profiles/)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)
    if args.gpus > 1 and env_world is None:
        # spawn the ranks here, before this process touches the GPU
        import torch.multiprocessing as mp
        mp.start_processes(_rank_main, args=(args, args.gpus, _free_port()), nprocs=args.gpus, join=True,
                           start_method="spawn")
        return
    run(args)


if __name__ == "__main__":
    main()
