"""One pass of fwd / pre / dq / dkdv per build on fresh buffers; reports non-finite
counts per output slice and the max difference between builds.
    python tools/nan_probe.py base=lib/libdiffattn.so g2=lib/libdiffattn_g2.so --shape B,H,hs,N,T"""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from differential_transformer_replication_amd import _lib  # noqa: E402
from ab_kernels import load, LIBDIR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("builds", nargs="+")
    ap.add_argument("--shape", default="8,8,128,3,4096")
    a = ap.parse_args()
    B, H, hs, N, T = (int(x) for x in a.shape.split(","))
    dv, nq = 2 * hs, H * N * hs
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, T, 2 * nq + H * dv, device=dev, generator=g).to(torch.bfloat16)
    do = torch.randn(B, T, H, dv, device=dev, generator=g).to(torch.bfloat16)
    coef = torch.randn(H, N, device=dev, generator=g) * 0.5
    coef[:, 0] = 1.0
    q = qkv[..., :nq].unflatten(-1, (H, N, hs))
    k = qkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
    v = qkv[..., 2 * nq:].unflatten(-1, (H, dv))
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = {}
    for b in a.builds:
        name, path = b.split("=", 1)
        lib = load(os.path.join(LIBDIR, path))
        o = torch.empty(B, T, H, dv, device=dev, dtype=torch.bfloat16)
        obr = torch.empty(N, B, T, H, dv, device=dev)
        lse = torch.empty(N, B, H, T, device=dev)
        dqkv = torch.zeros_like(qkv)
        dcoef = torch.empty(H, N, device=dev)
        delta = torch.empty(N, B, H, T, device=dev)
        obr_t = _lib.DtaTensor(obr.data_ptr(), *obr.stride()[1:4], obr.stride(0))
        fa = _lib.AttnFwdArgs(0, B, T, H, N, hs, dv, 1 / math.sqrt(hs), 0.0, _lib.tensor5(q), _lib.tensor5(k),
                              _lib.tensor5(v), _lib.tensor5(o), obr_t, lse.data_ptr(), coef.data_ptr())
        dq = dqkv[..., :nq].unflatten(-1, (H, N, hs))
        dk = dqkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
        dvv = dqkv[..., 2 * nq:].unflatten(-1, (H, dv))
        ba = _lib.AttnBwdArgs(0, B, T, H, N, hs, dv, 1 / math.sqrt(hs), 0.0, _lib.tensor5(q), _lib.tensor5(k),
                              _lib.tensor5(v), obr_t, lse.data_ptr(), coef.data_ptr(), _lib.tensor5(do),
                              _lib.tensor5(dq), _lib.tensor5(dk), _lib.tensor5(dvv), dcoef.data_ptr(),
                              delta.data_ptr(), None, _lib.BWD_PRE | _lib.BWD_DQ | _lib.BWD_DKDV, None)
        assert lib.dta_attn_fwd(fa, st) == 0 and lib.dta_attn_bwd(ba, st) == 0
        torch.cuda.synchronize()
        sl = {"o": o, "lse": lse, "dq": dq, "dk": dk, "dv": dvv, "dcoef": dcoef}
        print(name, {kk: int((~torch.isfinite(t.float())).sum()) for kk, t in sl.items()},
              {kk: float(t.float().abs().max()) for kk, t in sl.items()})
        outs[name] = sl
    base = a.builds[0].split("=")[0]
    for name in outs:
        print(name, "vs", base, {kk: float((outs[name][kk].float() - outs[base][kk].float()).abs().max())
                                 for kk in outs[base]})


if __name__ == "__main__":
    main()
