"""Average per-launch value of every collected counter, per attention kernel, from
rocprofv3 --pmc output directories, plus derived issue metrics.

    python tools/pmc_sq.py <dir> [<dir> ...] [--json out.json]

Derived (per launch; 1024 SIMDs, GRBM_GUI_ACTIVE summed over the 8 XCDs):
  valu_per_mfma   SQ_INSTS_VALU / SQ_INSTS_MFMA
  mfma_busy_frac  SQ_VALU_MFMA_BUSY_CYCLES / 1024 / (GRBM_GUI_ACTIVE / 8)
  wait_inst_frac  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (issue stalls: dependency / pipe busy)
  wait_any_frac   SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked in s_waitcnt / s_barrier)
  active_frac     SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  clock_ghz       GRBM_GUI_ACTIVE / 8 / kernel duration (End - Start of the same dispatches;
                  MI355X_MICROARCH.md 'DVFS give-back': the effective clock under load)
"""
import csv
import glob
import json
import sys
from collections import defaultdict

args = sys.argv[1:]
opts = {}
for flag in ("--json", "--lib-sha", "--shape"):
    if flag in args:
        i = args.index(flag)
        opts[flag] = args[i + 1]
        args = args[:i] + args[i + 2:]
out_json = opts.get("--json")
vals = defaultdict(list)
dur = defaultdict(list)          # kernel -> ns of the dispatches that carry GRBM_GUI_ACTIVE
for d in args:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            short = next((s for s in ("attn_fwd3", "attn_fwd2", "attn_fwd", "attn_dq2", "attn_dq", "attn_dkdv2", "attn_dkdv4", "attn_dkdv", "attn_bwd")
                          if s + "_kernel" in k), None)
            if short:
                vals[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("End_Timestamp"):
                    dur[short].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:12s} {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
per = defaultdict(dict)
for (k, c), v in vals.items():
    per[k][c] = sum(v) / len(v)
res = {}
for k, c in sorted(per.items()):
    d = {"counters": {n: round(x, 1) for n, x in sorted(c.items())}}
    g = lambda n: c.get(n)
    if g("SQ_INSTS_VALU") and g("SQ_INSTS_MFMA"):
        d["valu_per_mfma"] = round(g("SQ_INSTS_VALU") / g("SQ_INSTS_MFMA"), 2)
    if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
        d["mfma_busy_frac"] = round(g("SQ_VALU_MFMA_BUSY_CYCLES") / 1024 / (g("GRBM_GUI_ACTIVE") / 8), 4)
    for name, num in (("wait_inst_frac", "SQ_WAIT_INST_ANY"), ("wait_any_frac", "SQ_WAIT_ANY"),
                      ("active_frac", "SQ_ACTIVE_INST_ANY")):
        if g(num) and g("SQ_WAVE_CYCLES"):
            d[name] = round(g(num) / g("SQ_WAVE_CYCLES"), 4)
    if g("GRBM_GUI_ACTIVE") and dur.get(k):
        ns = sum(dur[k]) / len(dur[k])
        d["kernel_us"] = round(ns / 1e3, 1)
        d["clock_ghz"] = round(g("GRBM_GUI_ACTIVE") / 8 / ns, 3)
    res[k] = d
    print(k, {n: v for n, v in d.items() if n != "counters"})
if out_json:
    meta = {"source": "rocprofv3 --pmc, one counter group per pass, python3 bench.py --cpu-baseline off "
                      "--train-steps 0 --no-hbm --steps 2 --warmup 1 (tools/round_gpu.sh)"}
    if "--lib-sha" in opts:                      # the kernel build the counters were taken on (bench.py pairs by it)
        meta["lib_sha"] = opts["--lib-sha"]
    if "--shape" in opts:
        meta["shape"] = opts["--shape"]
    json.dump(dict(meta, kernels=res), open(out_json, "w"), indent=1)
