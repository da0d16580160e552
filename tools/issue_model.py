"""Single-wave issue model of one basic block of a hipcc -S listing (gfx950).

Reads the instructions of one loop body in program order and replays them for ONE wave
alone on a SIMD: in-order issue, a VGPR scoreboard, counted lgkmcnt waits, one matrix pipe.
The result is a cycle count per iteration that exposes serialised LDS-read -> wait -> MFMA
chains (each read's latency paid in full) long before a GPU run does; it is a
comparison tool for variants of one loop, not a prediction of wall time (the partner
wave on the SIMD, DMA and barriers are not modelled).

Costs (MI355X_MICROARCH.md 'Per-instruction cycle constants'): v_mfma_f32_32x32x16 holds
issue 8 cycles and the matrix pipe 32, result 64 cycles after issue (a dependent MFMA on
the same accumulator chains at the pipe rate); VALU 4 (transcendental 8), result after 8;
ds_read latency 64 (issue 4); s_nop N = N + 1; SALU 4.

    python tools/issue_model.py file.s <kernel-symbol-substring> <block-label>
"""
import re
import sys

from asm_loops import kernel_body

LDS_LAT, VALU_LAT, MFMA_LAT, MFMA_PIPE, MFMA_ISSUE = 64, 8, 64, 32, 8


def regs(tok):
    """VGPR indices named by one operand token (v5, v[4:7]); AGPRs count as VGPRs."""
    m = re.match(r"^[va]\[(\d+):(\d+)\]$", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"^[va](\d+)$", tok)
    return [int(m.group(1))] if m else []


def model(ins):
    t = 0                      # next issue cycle
    ready = {}                 # vgpr -> cycle its value is ready
    mfma_free = 0              # matrix pipe free at
    lds_q = []                 # completion times of outstanding LDS reads, in issue order
    last_mfma_dst = set()
    stall = {"lgkm": 0, "dep": 0, "pipe": 0}
    for line in ins:
        parts = line.replace(",", " ").split()
        op, ops = parts[0], parts[1:]
        if op.startswith("s_waitcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", line)
            if m:
                keep = int(m.group(1))
                while len(lds_q) > keep:
                    done = lds_q.pop(0)
                    if done > t:
                        stall["lgkm"] += done - t
                        t = done
            continue
        if op == "s_nop":
            t += int(ops[0]) + 1
            continue
        if op.startswith("s_"):
            t += 4 if op != "s_barrier" else 0
            continue
        dst = regs(ops[0]) if ops else []
        srcs = [r for o in ops[1:] for r in regs(o)]
        is_mfma = op.startswith("v_mfma")
        need = 0
        for r in srcs:
            rt = ready.get(r, 0)
            if is_mfma and r in last_mfma_dst:
                continue                   # accumulator chain: paced by the pipe
            need = max(need, rt)
        if need > t:
            stall["dep"] += need - t
            t = need
        if is_mfma:
            if mfma_free > t:
                stall["pipe"] += mfma_free - t
                t = mfma_free
            mfma_free = t + MFMA_PIPE
            for r in dst:
                ready[r] = t + MFMA_LAT
            last_mfma_dst = set(dst)
            t += MFMA_ISSUE
        elif op.startswith("ds_read"):
            lds_q.append(t + LDS_LAT)
            for r in dst:
                ready[r] = t + LDS_LAT
            t += 4
        elif op.startswith(("ds_write", "buffer_", "global_")):
            t += 8 if op.startswith("buffer_") else 4
        elif op.startswith("v_"):
            cost = 8 if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt")) else 4
            for r in dst:
                ready[r] = t + VALU_LAT
            t += cost
    return t, stall


def block(lines, label):
    out, on = [], False
    for l in lines:
        if re.match(r"^\.LBB\S+:", l):
            if on:
                break
            on = l.startswith(label + ":")
            continue
        s = l.strip()
        if on and s and not s.startswith((";", ".")):
            out.append(s.split(";")[0].strip())
    return out


def main():
    path, sym, label = sys.argv[1:4]
    ins = block(kernel_body(open(path).read().splitlines(), sym), label)
    cyc, stall = model(ins)
    nm = sum(1 for i in ins if i.startswith("v_mfma"))
    print(f"{label}: {len(ins)} instructions, {nm} MFMA, model {cyc} cycles "
          f"(MFMA floor {nm * MFMA_PIPE}); stalls {stall}")


if __name__ == "__main__":
    main()
