"""SURVEY 8(d) fidelity check of the CPU baseline (run in the build container,
where /root/reference exists; never on the GPU box).

Times, on this host's cores, one MultiHeadDiffAttention layer forward + backward
at B=1, T=4096, H=16, hs=64 (C=2048):
  * the reference module itself (imported read-only from /root/reference), and
  * the oracle's restatement of the same layer (oracle/diffattn_oracle.py),
and also bench.cpu_baseline() (the oracle's attention core alone, the number the
bench line reports).  The oracle must land within +-20% of the reference.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_fidelity.py profiles/r02_cpu_fidelity.json
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
B, T, H, HS = 1, 4096, 16, 64
C = 2 * H * HS
REPS = 2


def _time(fn, reps=REPS):
    fn()                                   # warm (allocator, threads)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sum(ts) / len(ts)


def main(out_path):
    sys.dont_write_bytecode = True
    threads = len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    sys.path.insert(0, "/root/reference")
    import diff_transformer as ref                              # the reference module, read-only
    from oracle import diffattn_oracle as orc
    import bench

    torch.manual_seed(0)
    m = ref.MultiHeadDiffAttention(H, HS, C, 0.0, T)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "lambda_" in n:
                p.normal_(0, 0.1)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, T, C, generator=g)
    dy = torch.randn(B, T, C, generator=g)

    def ref_step():
        xx = x.clone().requires_grad_(True)
        m(xx, 3).backward(dy)

    sd = {k: v.detach().clone().requires_grad_(v.is_floating_point() and "tril" not in k
                                              and "lambda_init" not in k)
          for k, v in m.state_dict().items()}

    def orc_step():
        xx = x.clone().requires_grad_(True)
        orc.multihead_diff_attention(xx, sd, H, 3, T).backward(dy)

    t_ref = _time(ref_step)
    t_orc = _time(orc_step)
    t0 = time.perf_counter()
    cb = bench.cpu_baseline()
    t_cb = time.perf_counter() - t0
    res = {
        "what": "MultiHeadDiffAttention fwd+bwd, B=1 T=4096 H=16 hs=64 C=2048, fp32, same weights and inputs",
        "host_threads": threads,
        "reference_s": round(t_ref, 3), "oracle_s": round(t_orc, 3),
        "oracle_over_reference": round(t_orc / t_ref, 3),
        "within_20pct": abs(t_orc / t_ref - 1) <= 0.2,
        "survey_6_reference_s": 1.494 + 1.780,
        "bench_cpu_baseline": cb, "bench_cpu_baseline_wall_s": round(t_cb, 2),
        "script": "tools/cpu_fidelity.py",
    }
    print(json.dumps(res, indent=1))
    if out_path:
        with open(out_path, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
