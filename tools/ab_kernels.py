"""One-process A/B of libdiffattn builds on the three attention kernels
(cdna_hip_programming.md 5.4 rule 24: interleaved rounds in ONE process).

Every build is loaded as its own ctypes handle (its own code object); the same
input tensors go through each build's dta_attn_fwd / dta_attn_bwd (DQ, DKDV
stages), timed with HIP events on the launch stream, ROUNDS x REPS, variants
interleaved.  Outputs of every variant are compared with the first build's.

    python tools/ab_kernels.py base=lib/libdiffattn.so v1=lib/libdiffattn_v1.so \
        [--shape B,H,hs,N,T] [--rounds 5] [--reps 10]
"""
import argparse
import ctypes
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from differential_transformer_replication_amd import _lib  # noqa: E402  (struct layouts only)

LIBDIR = os.path.join(ROOT, "differential_transformer_replication_amd")


def load(path):
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    lib.dta_attn_fwd.argtypes = [P(_lib.AttnFwdArgs), ctypes.c_void_p]
    lib.dta_attn_bwd.argtypes = [P(_lib.AttnBwdArgs), ctypes.c_void_p]
    lib.dta_attn_fwd.restype = lib.dta_attn_bwd.restype = ctypes.c_int
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("builds", nargs="+", help="name=path[@qcap,kcap] (path relative to the package dir)")
    ap.add_argument("--shape", default="8,16,64,2,4096")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--obr", choices=["f32", "f16"], default="f32", help="O_i storage (ABI 6 obr_dtype)")
    ap.add_argument("--dv", type=int, default=0, help="value width (default 2 * head size; head size for N = 1 control)")
    ap.add_argument("--mode", choices=["kernel", "step"], default="step",
                    help="kernel: each kernel REPS times back to back (its inputs stay in the 256 MB Infinity "
                         "Cache: optimistic for shapes whose operands fit); step: fwd, dq, dkdv in turn per rep, "
                         "as in a training step and bench.py (default)")
    args = ap.parse_args()
    B, H, hs, N, T = (int(x) for x in args.shape.split(","))
    dv = args.dv or 2 * hs
    dev = torch.device("cuda", 0)
    builds = []
    caps = {}
    for b in args.builds:
        name, path = b.split("=", 1)
        if "@" in path:                   # name=path@qcap,kcap: ABI 7 backward branch-group caps
            path, c = path.split("@", 1)
            caps[name] = tuple(int(x) for x in c.split(","))
        builds.append((name, load(path if os.path.isabs(path) else os.path.join(LIBDIR, path))))
    g = torch.Generator(device=dev).manual_seed(0)
    W = 2 * H * N * hs + H * dv
    nq = H * N * hs
    qkv = torch.randn(B, T, W, device=dev, generator=g).to(torch.bfloat16)
    do = torch.randn(B, T, H, dv, device=dev, generator=g).to(torch.bfloat16)
    coef = torch.randn(H, N, device=dev, generator=g) * 0.5
    coef[:, 0] = 1.0
    q = qkv[..., :nq].unflatten(-1, (H, N, hs))
    k = qkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
    v = qkv[..., 2 * nq:].unflatten(-1, (H, dv))
    stream = torch.cuda.current_stream(dev).cuda_stream
    scale = 1.0 / math.sqrt(hs)

    def bufs():
        o = torch.empty(B, T, H, dv, device=dev, dtype=torch.bfloat16)
        obr = torch.empty(N, B, T, H, dv, device=dev, dtype=torch.float16 if args.obr == "f16" else torch.float32)
        lse = torch.empty(N, B, H, T, device=dev)
        dqkv = torch.zeros_like(qkv)
        dcoef = torch.empty(H, N, device=dev)
        delta = torch.empty(N, B, H, T, device=dev)
        return o, obr, lse, dqkv, dcoef, delta

    state = {}
    for name, lib in builds:
        o, obr, lse, dqkv, dcoef, delta = bufs()
        obr_t = _lib.DtaTensor(obr.data_ptr(), *obr.stride()[1:4], obr.stride(0))
        fa = _lib.AttnFwdArgs(0, B, T, H, N, hs, dv, scale, 0.0, _lib.tensor5(q), _lib.tensor5(k), _lib.tensor5(v),
                              _lib.tensor5(o), obr_t, lse.data_ptr(), coef.data_ptr())
        fa.obr_dtype = 1 if args.obr == "f16" else 0
        dq = dqkv[..., :nq].unflatten(-1, (H, N, hs))
        dk = dqkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
        dvv = dqkv[..., 2 * nq:].unflatten(-1, (H, dv))
        ba = _lib.AttnBwdArgs(0, B, T, H, N, hs, dv, scale, 0.0, _lib.tensor5(q), _lib.tensor5(k), _lib.tensor5(v),
                              obr_t, lse.data_ptr(), coef.data_ptr(), _lib.tensor5(do), _lib.tensor5(dq),
                              _lib.tensor5(dk), _lib.tensor5(dvv), dcoef.data_ptr(), delta.data_ptr(), None,
                              _lib.BWD_PRE, None)
        ba.obr_dtype = fa.obr_dtype
        ba.group_max_dq, ba.group_max_dkdv = caps.get(name, (0, 0))
        # as ops._DiffAttention.backward: fixed-order d(coef) partials, and the fp32 dV
        # workspace when dK/dV runs in more than one branch group
        lib.dta_attn_bwd_dcoef_partial_bytes.argtypes = [ctypes.c_int32] * 4
        lib.dta_attn_bwd_dcoef_partial_bytes.restype = ctypes.c_size_t
        dcp = torch.empty(lib.dta_attn_bwd_dcoef_partial_bytes(B, T, H, N) // 4, device=dev)
        ba.dcoef_partial = dcp.data_ptr()
        keep = [dcp]
        if hasattr(lib, "dta_attn_bwd_dkdv_groups"):
            lib.dta_attn_bwd_dkdv_groups.argtypes = [ctypes.c_int32] * 5
            lib.dta_attn_bwd_dkdv_groups.restype = ctypes.c_int
            if lib.dta_attn_bwd_dkdv_groups(0, hs, N, dv, ba.group_max_dkdv) > 1:
                dv32 = torch.empty(B, T, H, dv, device=dev)
                ba.dv_f32 = dv32.data_ptr()
                keep.append(dv32)
        # ABI 8 lse_c workspace (as ops): builds without it ignore the field
        lsec = torch.empty(N, B, H, T, device=dev)
        ba.lse_c = lsec.data_ptr()
        keep.append(lsec)
        state[name] = (lib, fa, ba, (o, obr, lse, dqkv, dcoef), keep)

    def run(name, which):
        lib, fa, ba, _, _ = state[name]
        if which == "fwd":
            rc = lib.dta_attn_fwd(fa, stream)
        else:
            ba.stages = {"pre": _lib.BWD_PRE, "dq": _lib.BWD_DQ, "dkdv": _lib.BWD_DKDV}[which]
            rc = lib.dta_attn_bwd(ba, stream)
        if rc:
            raise RuntimeError(f"{name} {which}: rc {rc}")

    for name, _ in builds:                       # warm + produce outputs once
        for w in ("fwd", "pre", "dq", "dkdv"):
            run(name, w)
    torch.cuda.synchronize()
    base = builds[0][0]
    res = {n: {"fwd": [], "dq": [], "dkdv": []} for n, _ in builds}
    # the order rotates every round and each block's first launch is untimed: a fixed
    # order read the first build ~0.1 ms/step slow (profiles/r02_ab_sched_strategy.json)
    for r in range(args.rounds):
        for name, _ in builds[r % len(builds):] + builds[:r % len(builds)]:
            if args.mode == "step":
                for w in ("fwd", "pre", "dq", "dkdv"):       # untimed lead step
                    run(name, w)
                ev = {w: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                          for _ in range(args.reps)] for w in ("fwd", "dq", "dkdv")}
                for i in range(args.reps):
                    for w in ("fwd", "dq", "dkdv"):
                        if w == "dq":
                            run(name, "pre")
                        ev[w][i][0].record()
                        run(name, w)
                        ev[w][i][1].record()
                torch.cuda.synchronize()
                for w in ("fwd", "dq", "dkdv"):
                    res[name][w].extend(a.elapsed_time(b) for a, b in ev[w])
                continue
            for w in ("fwd", "dq", "dkdv"):
                if w == "dq":
                    run(name, "pre")
                run(name, w)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(args.reps)]
                for e0, e1 in ev:
                    if w == "dq":
                        run(name, "pre")
                    e0.record()
                    run(name, w)
                    e1.record()
                torch.cuda.synchronize()
                res[name][w].extend(a.elapsed_time(b) for a, b in ev)
    # correctness vs the first build (fresh single pass)
    out = {}
    for name, _ in builds:
        for w in ("fwd", "pre", "dq", "dkdv"):
            run(name, w)
    torch.cuda.synchronize()
    ref = state[base][3]
    for name, _ in builds:
        bo = state[name][3]
        diff = {lbl: float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-30))
                for lbl, a, b in zip(("o", "obr", "lse", "dqkv", "dcoef"), bo, ref)}
        med = {w: sorted(v)[len(v) // 2] for w, v in res[name].items()}
        mn = {w: min(v) for w, v in res[name].items()}
        out[name] = {"median_ms": {w: round(x, 4) for w, x in med.items()},
                     "min_ms": {w: round(x, 4) for w, x in mn.items()},
                     "sum_median_ms": round(sum(med.values()), 4), "rel_diff_vs_" + base: diff}
    print(json.dumps({"shape": dict(B=B, H=H, hs=hs, N=N, T=T), "mode": args.mode, "rounds": args.rounds, "reps": args.reps,
                      "builds": out}, indent=1))


if __name__ == "__main__":
    main()
