"""Per-launch HBM traffic of the attention kernels from two rocprofv3 passes
(--pmc FETCH_SIZE, --pmc WRITE_SIZE; tools/profile_round.sh) -> profiles JSON.

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of 16-B/lane streaming
reads (MI355X_MICROARCH.md, HBM section).  Usage:
    python tools/pmc_summary.py gpurun_out/<tag> profiles/<tag>_pmc_traffic.json
"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

NAMES = {"attn_fwd_kernel": "attn_fwd", "attn_dq_kernel": "attn_bwd_dq", "attn_dkdv_kernel": "attn_bwd_dkdv",
         "attn_dq2_kernel": "attn_bwd_dq", "attn_dkdv2_kernel": "attn_bwd_dkdv",
         "attn_fwd2_kernel": "attn_fwd", "attn_fwd3_kernel": "attn_fwd",
         "decode_split_kernel": "decode_split", "decode_combine_kernel": "decode_combine",
         "ln_fwd_kernel": "ln_fwd", "ln_bwd_kernel": "ln_bwd", "ln_bwd_rb_kernel": "ln_bwd", "rope_kernel": "rope"}


def per_kernel(path, counter):
    vals = defaultdict(list)
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for key, short in NAMES.items():
                if key in r["Kernel_Name"]:
                    vals[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main(src, dst, shape=None):
    fetch = per_kernel(src + "/pmc_fetch", "FETCH_SIZE")
    write = per_kernel(src + "/pmc_write", "WRITE_SIZE")
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, python3 bench.py "
                     f"--cpu-baseline off --steps 3 --warmup 1 (tools/profile_round.sh, {src})",
           "units": "bytes per launch; FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE doubled (gfx950: counts half "
                    "the bytes of 16B/lane streaming reads, MI355X_MICROARCH.md HBM section)",
           "kernels": {}}
    # the kernel build these counters were taken on: bench.py reports the traffic only
    # while the library it runs is this same build
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "differential_transformer_replication_amd", "lib", "libdiffattn.so")
    with open(lib, "rb") as fh:
        out["lib_sha"] = hashlib.sha256(fh.read()).hexdigest()[:16]
    if shape:
        # the attention workload these launches ran at (bench.shape_key); ln_* / rope are at
        # their fixed hbm_bench shapes (bench.py hbm_bench docstring)
        out["shape"] = shape
    for k in NAMES.values():
        if k not in fetch or k not in write:
            continue
        rd = int(fetch[k] * 1024 * 2)
        wr = int(write[k] * 1024)
        out["kernels"][k] = {"fetch_size_kib_raw": round(fetch[k], 1), "write_size_kib": round(write[k], 1),
                             "read_bytes": rd, "write_bytes": wr, "traffic_bytes": rd + wr}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out["kernels"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
