"""Audit hand-written (inline asm) MFMAs in a hipcc -save-temps .s for the VALU-write -> MFMA-read
hazard the compiler does not pad across an asm boundary: an MFMA inside ;;#ASMSTART/;;#ASMEND whose
A/B/C VGPR (or AGPR) operand was written by a VALU / v_accvgpr instruction fewer than NEED wait
states earlier (s_nop N counts N+1 states, every other instruction 1).

    python scripts/diag/asm_mfma_hazards.py /tmp/attn_kernels-hip-amdgcn-amd-amdhsa-gfx950.s [--need 2]"""
import argparse
import re

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out |= {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("s")
    ap.add_argument("--need", type=int, default=2)
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    func, in_asm, hist, bad = None, False, [], 0
    for ln in open(a.s):
        t = ln.split(";")[0].strip() if not ln.strip().startswith(";;#ASM") else ln.strip()
        if re.match(r"^_Z\w+:$", t):
            func, hist = t[:-1], []
            continue
        if t == ";;#ASMSTART":
            in_asm = True
            continue
        if t == ";;#ASMEND":
            in_asm = False
            continue
        if not t or t.endswith(":") or t.startswith("."):
            if t.endswith(":"):
                hist = []                    # a label: do not reason across control flow
            continue
        op = t.split()[0]
        if op.startswith("v_mfma") and in_asm and func and a.kernel in func:
            ops = t.split(None, 1)[1].split(",")
            srcs = regs(",".join(ops[1:]))
            states = 0
            for hop, hdst, hn in reversed(hist):
                if states >= a.need:
                    break
                if hdst & srcs and not hop.startswith(("v_mfma", "ds_", "global_", "buffer_")):
                    print(f"{func[:60]}: {t}  <- {hop} {sorted(hdst & srcs)[:4]} after {states} states")
                    bad += 1
                    break
                states += hn
        n = 1
        if op == "s_nop":
            n = int(t.split()[1], 0) + 1
        dst = set()
        if op.startswith("v_") and "," in t:
            dst = regs(t.split(None, 1)[1].split(",")[0])
        hist.append((op, dst, n))
        hist = hist[-16:]
    print("hazards:", bad)


if __name__ == "__main__":
    main()
