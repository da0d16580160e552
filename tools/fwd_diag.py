"""Forward of one build against another (same process, two ctypes handles): where the
outputs differ -- per branch, per query row block of 32, per 32-column block of O_i, and
the LSE -- for debugging a new forward kernel.

    DTA_FWD3=1 python tools/fwd_diag.py new=lib/libdiffattn.so ref=lib/libdiffattn_nodq2.so \
        [--shapes 2,2,64,2,129 ...]
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from differential_transformer_replication_amd import _lib  # noqa: E402
from ab_kernels import load, LIBDIR  # noqa: E402


def run_fwd(lib, q, k, v, coef, B, T, H, N, hs, dv, dev, stream):
    o = torch.zeros(B, T, H, dv, device=dev, dtype=torch.bfloat16)
    obr = torch.zeros(N, B, T, H, dv, device=dev, dtype=torch.float32)
    lse = torch.zeros(N, B, H, T, device=dev)
    obr_t = _lib.DtaTensor(obr.data_ptr(), *obr.stride()[1:4], obr.stride(0))
    fa = _lib.AttnFwdArgs(0, B, T, H, N, hs, dv, 1.0 / math.sqrt(hs), 0.0, _lib.tensor5(q), _lib.tensor5(k),
                          _lib.tensor5(v), _lib.tensor5(o), obr_t, lse.data_ptr(), coef.data_ptr())
    rc = lib.dta_attn_fwd(fa, stream)
    torch.cuda.synchronize()
    if rc:
        raise RuntimeError(f"rc {rc}")
    return o.float(), obr, lse


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("builds", nargs=2)
    ap.add_argument("--shapes", nargs="+", default=["2,2,64,2,129", "1,1,64,2,256", "2,4,64,2,1000"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    libs = [(b.split("=", 1)[0], load(os.path.join(LIBDIR, b.split("=", 1)[1]))) for b in args.builds]
    stream = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    for sh in args.shapes:
        B, H, hs, N, T = (int(x) for x in sh.split(","))
        dv = 2 * hs
        g = torch.Generator(device=dev).manual_seed(0)
        nq = H * N * hs
        qkv = torch.randn(B, T, 2 * nq + H * dv, device=dev, generator=g).to(torch.bfloat16)
        q = qkv[..., :nq].unflatten(-1, (H, N, hs))
        k = qkv[..., nq:2 * nq].unflatten(-1, (H, N, hs))
        v = qkv[..., 2 * nq:].unflatten(-1, (H, dv))
        coef = torch.randn(H, N, device=dev, generator=g) * 0.5
        coef[:, 0] = 1.0
        outs = [run_fwd(lib, q, k, v, coef, B, T, H, N, hs, dv, dev, stream) for _, lib in libs]
        (o1, b1, l1), (o2, b2, l2) = outs
        scale = b2.abs().max().item()
        d = torch.nan_to_num((b1 - b2).abs() / scale, nan=9.0)  # [N][B][T][H][dv]
        nrb = (T + 31) // 32
        per_rows = [round(d[:, :, 32 * r:32 * r + 32].max().item(), 4) for r in range(nrb)]
        per_branch = [round(d[i].max().item(), 4) for i in range(N)]
        per_col = [round(d[..., 32 * c:32 * c + 32].max().item(), 4) for c in range(dv // 32)]
        per_row_in_blk = [round(d[:, :, [t for t in range(T) if t % 32 == r]].max().item(), 4) for r in range(32)]
        dl = (l1 - l2).abs()                                      # [N][B][H][T]
        lse_rows = [round(dl[..., 32 * r:32 * r + 32].max().item(), 4) for r in range(nrb)]
        nanrows = sorted(set(torch.nonzero(~torch.isfinite(b1).all(dim=-1).all(dim=-1).all(dim=0).all(dim=0))[:, 0].tolist())) if False else \
            sorted(set(torch.nonzero((~torch.isfinite(b1)).any(dim=-1).any(dim=-1).any(dim=0).any(dim=0))[:, 0].tolist()))
        d = torch.nan_to_num(d, nan=9.0)
        res[sh] = {"nan_rows": nanrows[:40], "n_nan_rows": len(nanrows),
                   "o": round(((o1 - o2).abs().max() / o2.abs().max()).item(), 5), "obr_branch": per_branch,
                   "obr_rowblk": per_rows, "obr_colblk": per_col, "obr_row_mod32": per_row_in_blk,
                   "lse_rowblk": lse_rows, "finite": bool(torch.isfinite(b1).all().item())}
        print(sh, json.dumps(res[sh]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
