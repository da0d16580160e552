"""Per-(kernel, grid) rocprofv3 summary.

rocprofv3's own --stats groups launches by kernel name only, so one kernel instance that
runs at several shapes in the same process (bench.py's cfg2 core and its cfg3 legs) gets a
mean over all of them.  This groups the kernel trace by (kernel, grid, workgroup) instead:

    python tools/kernel_stats_by_shape.py <run_kernel_trace.csv> <out.csv> [--top 40]

Columns: kernel (demangled-ish short name), full mangled name, grid x/y/z, workgroup size,
calls, mean / min / max / total duration (us).  Rows sorted by total time.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.match(r"_ZN3dta\d+(\w+?_kernel)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    groups = defaultdict(list)
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            # Grid_Size_* are in work-items: report workgroups
            gx = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            gy = int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_Y"]))
            gz = int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_Z"]))
            key = (r["Kernel_Name"], gx, gy, gz, wg)
            groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    rows = []
    for (name, gx, gy, gz, wg), d in groups.items():
        rows.append([short(name), gx, gy, gz, wg, len(d), sum(d) / len(d), min(d), max(d), sum(d), name])
    rows.sort(key=lambda r: -r[9])
    with open(a.out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "grid_x", "grid_y", "grid_z", "wg_threads", "calls", "mean_us", "min_us", "max_us",
                    "total_us", "mangled"])
        for r in rows[:a.top]:
            w.writerow(r[:6] + [f"{x:.1f}" for x in r[6:10]] + [r[10]])
    for r in rows[:12]:
        print(f"{r[0]:28s} grid {r[1]}x{r[2]}x{r[3]} wg {r[4]:4d} calls {r[5]:3d} mean {r[6]:9.1f} us")


if __name__ == "__main__":
    main()
