"""Per-basic-block instruction mix of one kernel in a hipcc -S listing, to read the
main loops' VALU / MFMA / LDS / SALU counts.   python tools/asm_loops.py file.s <kernel-symbol-substring> [min_mfma]"""
import re
import sys
from collections import Counter


def kernel_body(lines, sym):
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith("_Z") and sym in l and l.rstrip().endswith(":") or (
                start is None and l.startswith("_Z") and sym in l and ": ;" in l):
            start = i
        elif start is not None and l.startswith("\t.size") or (start is not None and l.startswith(".Lfunc_end")):
            return lines[start:i]
    return lines[start:] if start is not None else []


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("v_"):
        if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt")):
            return "trans"
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_barrier",)):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    min_mfma = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    body = kernel_body(open(path).read().splitlines(), sym)
    blocks, cur, name = [], [], "entry"
    for l in body:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), []
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        cur.append(s.split()[0])
    blocks.append((name, cur))
    tot = Counter()
    for name, ins in blocks:
        c = Counter(classify(o) for o in ins)
        tot.update(c)
        if c["mfma"] >= min_mfma:
            valu_ops = Counter(o for o in ins if classify(o) in ("valu", "trans"))
            print(f"{name}: n={len(ins)} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
            print("   top valu:", ", ".join(f"{k}:{v}" for k, v in valu_ops.most_common(18)))
            salu = Counter(o for o in ins if classify(o) == "salu")
            print("   top salu:", ", ".join(f"{k}:{v}" for k, v in salu.most_common(10)))
    print("kernel total:", " ".join(f"{k}={v}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
