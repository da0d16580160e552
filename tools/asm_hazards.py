"""Static check of the kernels whose accumulators are written by inline-asm MFMAs
(mfma_agpr: attn_fwd3 / attn_dq2 / attn_dkdv2).

The compiler does not see an asm MFMA's latency: it treats the accumulator as written
when the asm statement issues.  Any instruction it places soon after that reads those
AGPRs -- a scratch spill, an allocator copy (v_accvgpr_mov), a v_accvgpr_read -- reads
the value from before the MFMA.  This walks the ISA of every such kernel in straight-line
order and reports reads of an asm-MFMA destination within 18 issue cycles of it (the
32x32x16 bf16 MFMA's result latency in wait states), and every scratch access.

    python tools/asm_hazards.py <file.s>            (exit status 1 on any finding)
    python tools/asm_hazards.py --build [unit]      (hipcc -S of csrc/<unit>.hip first)
"""
import os
import re
import subprocess
import sys

KERNELS = re.compile(r"^(_ZN3dta\d+attn_(?:fwd3|dq2|dkdv2)_kernel\w*):", re.M)
STORES = ("scratch_store", "global_store", "buffer_store", "ds_write")
WAIT_STATES = 18


def scan(text):
    out = {}
    for m in KERNELS.finditer(text):
        name = m.group(1)
        end = text.index(".Lfunc_end", m.end())
        lines = [ln.split(";")[0].strip() for ln in text[m.end():end].split("\n")]
        lines = [ln for ln in lines if ln and not ln.startswith(".") and not ln.endswith(":")]
        cyc, written, hazards, scratch = 0, {}, [], 0
        reading, read_at = set(), 0   # VGPRs an asm MFMA (AGPR destination) may still be reading
        for ln in lines:
            parts = ln.replace(",", " ").split()
            op = parts[0]
            if op.startswith("scratch_"):
                scratch += 1
            cyc += int(parts[1]) + 1 if op == "s_nop" else 1
            if op.startswith(("s_waitcnt", "s_barrier")):
                cyc += 16                  # at least that long, in practice far longer
            if reading and cyc - read_at > WAIT_STATES:
                reading = set()            # the MFMA has read its operands by now
            if op.startswith("v_mfma"):
                reading, read_at = set(), cyc
                d = re.match(r"a\[(\d+):(\d+)\]", parts[1])
                if d:
                    for r in range(int(d.group(1)), int(d.group(2)) + 1):
                        written[r] = cyc
                    for o in parts[2:4]:
                        v = re.match(r"v\[(\d+):(\d+)\]$", o)
                        if v:
                            reading.update(range(int(v.group(1)), int(v.group(2)) + 1))
                continue
            # write-after-read: a VGPR source of the last asm MFMA overwritten before the
            # next MFMA issues (LDS reads excepted: their data returns >= 64 cycles later)
            if reading and op.startswith("v_") and len(parts) > 1:
                v = re.match(r"v(\d+)$", parts[1]) or re.match(r"v\[(\d+):(\d+)\]$", parts[1])
                if v:
                    regs = [int(v.group(1))] if v.lastindex == 1 else range(int(v.group(1)), int(v.group(2)) + 1)
                    if any(r in reading for r in regs):
                        hazards.append("WAR " + ln)
            for o in (parts[1:] if op.startswith(STORES) else parts[2:]):
                a = re.match(r"a(\d+)$", o) or re.match(r"a\[(\d+):(\d+)\]$", o)
                if not a:
                    continue
                regs = [int(a.group(1))] if a.lastindex == 1 else range(int(a.group(1)), int(a.group(2)) + 1)
                if any(r in written and cyc - written[r] < WAIT_STATES for r in regs):
                    hazards.append(ln)
                    break
        out[name] = {"hazards": hazards, "scratch": scratch}
    return out


def build_asm(unit="attn_bf16_dq2"):
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "differential_transformer_replication_amd", "csrc")
    dst = os.path.join("/tmp", f"dta_{unit}_{os.getpid()}.s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
           "-fno-honor-nans", "-fno-slp-vectorize", "-w", "--cuda-device-only", "-S",
           os.path.join(csrc, unit + ".hip"), "-o", dst]
    if unit == "attn_bf16_dq2":
        cmd[1:1] = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
    subprocess.run(cmd, check=True, cwd=csrc)
    with open(dst) as f:
        text = f.read()
    os.unlink(dst)
    return text


def main():
    args = sys.argv[1:]
    text = build_asm(*(args[1:2] or [])) if args and args[0] == "--build" else open(args[0]).read()
    res = scan(text)
    bad = 0
    for name, r in sorted(res.items()):
        flag = "OK " if not r["hazards"] and not r["scratch"] else "BAD"
        bad += flag == "BAD"
        print(f"{flag} {name[:72]:72s} hazards {len(r['hazards'])} scratch {r['scratch']}")
        for h in r["hazards"][:3]:
            print("      ", h)
    sys.exit(1 if bad or not res else 0)


if __name__ == "__main__":
    main()
