"""One-process A/B of libdiffattn builds on the LayerNorm kernels at the cfg2
GroupLayerNorm shape (32768 rows x 2048, bf16): dta_ln_fwd and dta_ln_bwd (with the
ordered dw/db reduce), HIP events, rounds interleaved; dx, y and dw/db compared with the first build.
    python tools/ab_ln.py base=lib/libdiffattn_x.so new=lib/libdiffattn.so"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from differential_transformer_replication_amd import _lib  # noqa: E402


def main():
    builds = [a.split("=", 1) for a in sys.argv[1:]]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    rows, C = 8 * 4096, 2048
    x = torch.randn(rows, C, device=dev, dtype=torch.bfloat16, generator=g)
    w = torch.ones(C, device=dev) + 0.1 * torch.randn(C, device=dev, generator=g)
    b = 0.1 * torch.randn(C, device=dev, generator=g)
    dy = torch.randn(rows, C, device=dev, dtype=torch.bfloat16, generator=g)
    y, dx = torch.empty_like(x), torch.empty_like(x)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = {}
    for name, path in builds:
        lib = ctypes.CDLL(os.path.join(ROOT, "differential_transformer_replication_amd", path))
        lib.dta_ln_fwd.argtypes = lib.dta_ln_bwd.argtypes = [ctypes.POINTER(_lib.LnArgs), ctypes.c_void_p]
        lib.dta_ln_bwd_workspace_bytes.argtypes = [ctypes.c_int64] * 2
        lib.dta_ln_bwd_workspace_bytes.restype = ctypes.c_size_t
        lib.dta_rope.argtypes = [ctypes.POINTER(_lib.RopeArgs), ctypes.c_void_p]
        libs[name] = lib
    # RoPE of every Q_i / K_i at cfg3 (bench.py hbm_bench's rope shape)
    Br, Tr, H2, Nr, hr = 16, 2048, 12, 3, 64
    rsrc = torch.randn(Br, Tr, H2, Nr, hr, device=dev, generator=g).to(torch.bfloat16)
    rdst = torch.empty_like(rsrc)
    from differential_transformer_replication_amd.Ndiff_transformer import precompute_freqs_cis
    table = torch.view_as_real(precompute_freqs_cis(hr, Tr)).to(dev).contiguous()
    ra = _lib.RopeArgs(_lib.DTA_BF16, Br, Tr, H2, Nr, hr, 0, 0, _lib.tensor5(rsrc), _lib.tensor5(rdst), table.data_ptr())
    part = torch.empty(max(l.dta_ln_bwd_workspace_bytes(rows, C) for l in libs.values()) // 4, device=dev)
    fa = _lib.LnArgs(_lib.DTA_BF16, rows, C, 1e-5, 0.2, x.data_ptr(), C, y.data_ptr(), C, w.data_ptr(),
                     b.data_ptr(), mean.data_ptr(), rstd.data_ptr(), None, 0, None, 0, None, None)
    ba = _lib.LnArgs(_lib.DTA_BF16, rows, C, 1e-5, 0.2, x.data_ptr(), C, None, 0, w.data_ptr(), None,
                     mean.data_ptr(), rstd.data_ptr(), dy.data_ptr(), C, dx.data_ptr(), C, dw.data_ptr(),
                     db.data_ptr(), part.data_ptr())
    times = {n: {"fwd": [], "bwd": [], "rope": []} for n in libs}
    ref = None
    for rnd in range(6):
        for n, lib in libs.items():
            for kind, fn in (("fwd", lambda: lib.dta_ln_fwd(fa, stream)), ("bwd", lambda: lib.dta_ln_bwd(ba, stream)),
                             ("rope", lambda: lib.dta_rope(ra, stream))):
                for _ in range(2):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[n][kind].append(e0.elapsed_time(e1) / 10 * 1e3)
            if rnd == 0:
                dw.zero_(); db.zero_()              # one backward from zero: dw / db comparable
                lib.dta_ln_bwd(ba, stream)
                torch.cuda.synchronize()
                if ref is None:
                    ref = (dx.clone(), y.clone(), rdst.clone(), dw.clone(), db.clone())
                else:
                    times[n]["dx_equal"] = bool(torch.equal(ref[0], dx))
                    times[n]["y_equal"] = bool(torch.equal(ref[1], y))
                    times[n]["rope_equal"] = bool(torch.equal(ref[2], rdst))
                    times[n]["dw_db_equal"] = bool(torch.equal(ref[3], dw) and torch.equal(ref[4], db))
    out = {}
    for n, d in times.items():
        out[n] = {k: (sorted(v)[len(v) // 2] if isinstance(v, list) else v) for k, v in d.items()}
        out[n]["bwd_TBps"] = 3 * rows * C * 2 / out[n]["bwd"] / 1e6
        out[n]["fwd_TBps"] = 2 * rows * C * 2 / out[n]["fwd"] / 1e6
        out[n]["rope_TBps"] = 2 * rsrc.numel() * 2 / out[n]["rope"] / 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()
