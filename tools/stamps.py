"""Cycle shares of the forward and dK/dV tile loops from a DTA_STAMPS=1 build
(tools/build_variant.sh stamps "-DDTA_STAMPS=1").  Read the SHARES, not the
length: the stamps' lgkmcnt(0) waits serialise LDS reads.

    python tools/stamps.py lib/libdiffattn_stamps.so [--shape B,H,hs,N,T]
"""
import argparse
import ctypes
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from differential_transformer_replication_amd import _lib  # noqa: E402

FWD_SEGS = ["dma_issue", "qk_softmax", "pv", "wait_vm", "barrier", "tail", "-", "loop_top"]
DKDV_SEGS = ["dma_issue", "compute(dP,S,dS,dK,dV)", "wait_vm", "barrier", "-", "-", "-", "-"]
DQ_SEGS = ["dma_issue", "dP", "branches(S,dS,dQ)", "wait_vm", "barrier", "-", "-", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--shape", default="8,16,64,2,4096")
    args = ap.parse_args()
    B, H, hs, N, T = (int(x) for x in args.shape.split(","))
    dv = 2 * hs
    path = args.lib if os.path.isabs(args.lib) else os.path.join(ROOT, "differential_transformer_replication_amd", args.lib)
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    lib.dta_attn_fwd.argtypes = [P(_lib.AttnFwdArgs), ctypes.c_void_p]
    lib.dta_attn_bwd.argtypes = [P(_lib.AttnBwdArgs), ctypes.c_void_p]
    lib.dta_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda", 0)
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
    o = torch.empty(B, T, H, dv, device=dev, dtype=torch.bfloat16)
    obr = torch.empty(N, B, T, H, dv, device=dev, dtype=torch.float32)
    lse = torch.empty(N, B, H, T, device=dev)
    dqkv = torch.zeros_like(qkv)
    dcoef = torch.empty(H, N, device=dev)
    delta = torch.empty(N, B, H, T, device=dev)
    obr_t = _lib.DtaTensor(obr.data_ptr(), *obr.stride()[1:4], obr.stride(0))
    stream = torch.cuda.current_stream(dev).cuda_stream
    fa = _lib.AttnFwdArgs(0, B, T, H, N, hs, dv, 1 / math.sqrt(hs), 0.0, _lib.tensor5(q), _lib.tensor5(k),
                          _lib.tensor5(v), _lib.tensor5(o), obr_t, lse.data_ptr(), coef.data_ptr())
    dq = dqkv[..., :nq].unflatten(-1, (H, N, hs))
    dk = dqkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
    dvv = dqkv[..., 2 * nq:].unflatten(-1, (H, dv))
    ba = _lib.AttnBwdArgs(0, B, T, H, N, hs, dv, 1 / math.sqrt(hs), 0.0, _lib.tensor5(q), _lib.tensor5(k),
                          _lib.tensor5(v), obr_t, lse.data_ptr(), coef.data_ptr(), _lib.tensor5(do),
                          _lib.tensor5(dq), _lib.tensor5(dk), _lib.tensor5(dvv), dcoef.data_ptr(),
                          delta.data_ptr(), None, 0, None)
    out = {}
    nbytes = 8 << 20
    for which in ("fwd", "dq", "dkdv"):
        # dq: the PRE + DQ stages only (the DKDV stage would overwrite the per-wave slots)
        ba.stages = _lib.BWD_PRE | _lib.BWD_DQ if which == "dq" else 0
        for _ in range(30):                      # >= 2 s of back-to-back launches would be ideal; shares only
            assert (lib.dta_attn_fwd(fa, stream) if which == "fwd" else lib.dta_attn_bwd(ba, stream)) == 0
        torch.cuda.synchronize()
        buf = np.zeros(nbytes // 8, dtype=np.uint64)
        assert lib.dta_debug_stamps(buf.ctypes.data, nbytes) == 0
        st = buf.reshape(-1, 8)
        st = st[st.sum(1) > 0].astype(np.float64)
        names = {"fwd": FWD_SEGS, "dq": DQ_SEGS, "dkdv": DKDV_SEGS}[which]
        tot = st.sum(0)
        out[which] = {"waves": int(st.shape[0]),
                      "share": {n: round(float(x / tot.sum()), 4) for n, x in zip(names, tot) if n != "-"},
                      "mean_cycles_per_wave": {n: round(float(x / st.shape[0])) for n, x in zip(names, tot) if n != "-"}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
