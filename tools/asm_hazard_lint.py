"""Hazard lint for the inline-asm MFMAs of a hipcc --save-temps .s file (cdna_hip_programming.md
§5.7: hipcc pads no hazard whose producer or consumer is inside an asm statement).

For every `v_mfma_*` between ;;#ASMSTART / ;;#ASMEND, report a VALU instruction (v_*, not an MFMA)
among the N instructions before it that writes one of the MFMA's source registers (VGPR or AGPR):
such a write needs >= 2 wait states before an MFMA reads it.  usage: asm_hazard_lint.py FILE.s [N]
exit 1 when a hazard is found."""
import re
import sys


def regs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {tok} if m else set()


def main():
    path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
    lines = [l.split(";")[0].strip() for l in open(path)]
    insts, in_asm = [], False
    for raw in open(path):
        t = raw.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        t = t.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        insts.append((t, in_asm))
    bad = 0
    for i, (t, asm) in enumerate(insts):
        if not (asm and t.startswith("v_mfma")):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        srcs = set().union(*(regs(o) for o in ops[1:]))
        for j in range(max(0, i - n), i):
            p, _ = insts[j]
            if p.startswith("s_nop"):
                break
            if not p.startswith("v_") or p.startswith("v_mfma"):
                continue
            dst = regs(p.split(None, 1)[1].split(",")[0].strip()) if " " in p else set()
            if dst & srcs:
                print(f"hazard: '{p}' -> '{t}'")
                bad += 1
    print(f"{path}: {bad} hazard(s)")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
