"""issue_model.py's replay with the per-instruction stalls printed (> min cycles)."""
import re
import sys

import issue_model as M
from asm_loops import kernel_body


def main():
    path, sym, label = sys.argv[1:4]
    lim = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    ins = M.block(kernel_body(open(path).read().splitlines(), sym), label)
    t, ready, mfma_free, lds_q, last = 0, {}, 0, [], set()
    for idx, line in enumerate(ins):
        parts = line.replace(",", " ").split()
        op, ops = parts[0], parts[1:]
        t0 = t
        if op.startswith("s_waitcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", line)
            if m:
                while len(lds_q) > int(m.group(1)):
                    t = max(t, lds_q.pop(0))
        elif op == "s_nop":
            t += int(ops[0]) + 1
        elif op.startswith("s_"):
            t += 4
        else:
            dst = M.regs(ops[0]) if ops else []
            srcs = [r for o in ops[1:] for r in M.regs(o)]
            mf = op.startswith("v_mfma")
            need = max([ready.get(r, 0) for r in srcs if not (mf and r in last)] + [0])
            t = max(t, need)
            if mf:
                t = max(t, mfma_free)
                mfma_free = t + M.MFMA_PIPE
                for r in dst:
                    ready[r] = t + M.MFMA_LAT
                last = set(dst)
                t += M.MFMA_ISSUE
            elif op.startswith("ds_read"):
                lds_q.append(t + M.LDS_LAT)
                for r in dst:
                    ready[r] = t + M.LDS_LAT
                t += 4
            elif op.startswith("v_"):
                for r in dst:
                    ready[r] = t + M.VALU_LAT
                t += 8 if op.startswith(("v_exp", "v_log", "v_rcp")) else 4
            else:
                t += 4
        if t - t0 > lim:
            print(f"{idx:4d} t={t0:5d} +{t - t0:3d}  {line}")
    print("total", t)


if __name__ == "__main__":
    main()
