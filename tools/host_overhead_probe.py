"""Where the bench's cfg3 core step loses time outside its kernels (verdict round 5, Weak #6).

For a shape, K steps of ops.diff_attention forward + backward exactly as bench.core_run runs
them, three ways:
  host_ms   time to ENQUEUE one step (no synchronize inside the loop): the Python / autograd /
            ctypes / allocator work per step on the host;
  wall_ms   wall time per step with a synchronize at both ends (the bench's number);
  gpu_ms    the sum of the attention kernels' HIP-event times per step (ops.TIMER);
  + the same wall time with ops.TIMER off (its 6 events per step) and with the step captured
    in a HIP graph (host work removed entirely).
If wall ~ host > gpu, the loop is host-bound and the kernels idle between launches.

    python tools/host_overhead_probe.py [--shape B,H,hs,N,T] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from differential_transformer_replication_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16,6,64,3,2048")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    B, H, hs, N, T = (int(x) for x in args.shape.split(","))
    dv = 2 * hs
    dev = torch.device("cuda", 0)
    W = ops.packed_width(H, N, hs, dv)
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, T, W, device=dev, dtype=torch.bfloat16, generator=g).requires_grad_(True)
    do = torch.randn(B, T, H * dv, device=dev, dtype=torch.bfloat16, generator=g)
    coef = bench._coefficients(H, N, hs, dev)

    def step():
        qkv.grad = None
        ops.diff_attention(qkv, coef, H, N, hs, dv=dv).backward(do)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    res = {"shape": dict(B=B, H=H, hs=hs, N=N, T=T), "steps": args.steps}
    # host enqueue time and wall time, TIMER on (as the bench)
    ops.TIMER.start()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ops.TIMER.stop()
    kt = ops.TIMER.mean_ms()
    res["timer_on"] = {"host_ms": round((t1 - t0) * 1e3 / args.steps, 4), "wall_ms": round((t2 - t0) * 1e3 / args.steps, 4),
                       "gpu_ms": round(sum(v[0] * v[1] for v in kt.values()) / args.steps, 4),
                       "kernels": {k: round(v[0], 4) for k, v in kt.items()}}
    # TIMER off
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res["timer_off"] = {"host_ms": round((t1 - t0) * 1e3 / args.steps, 4), "wall_ms": round((t2 - t0) * 1e3 / args.steps, 4)}
    # graph-captured step (no host work per step)
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        qkv.grad = None
        with torch.cuda.graph(graph):
            ops.diff_attention(qkv, coef, H, N, hs, dv=dv).backward(do)
        graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            graph.replay()
        torch.cuda.synchronize()
        res["graph"] = {"wall_ms": round((time.perf_counter() - t0) * 1e3 / args.steps, 4)}
    except Exception as e:          # report, do not fail the probe
        res["graph"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
