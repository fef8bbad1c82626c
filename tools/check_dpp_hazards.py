"""Static check of the VALU-write -> DPP-read hazard in a hipcc -S listing (gfx9: a DPP
instruction reading a VGPR written by a VALU instruction needs 2 wait states in between).

The IPM kernel emits its DPP instructions from inline asm, whose hazards hipcc does not see;
this walks back from every DPP instruction over the straight-line code before it and fails if a
VALU write of the DPP source register lies within 2 wait states (s_nop N counts N+1, any other
instruction 1).  A label ends the walk (the predecessor is then the fall-through path only, which
is what the unrolled kernels have; a loop back edge is checked at its own DPP).

    python tools/check_dpp_hazards.py file.s      (exit status 1 on a hazard)
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok):
    m = REG.fullmatch(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return {int(m.group(3))}


def operands(line):
    parts = line.split(None, 1)
    if len(parts) < 2:
        return parts[0], []
    ops = [o.strip() for o in parts[1].split(",")]
    return parts[0], ops


def check(lines):
    bad = []
    insts = []   # (lineno, text) of instructions and labels, comments dropped
    for n, l in enumerate(lines):
        t = l.split(";")[0].strip()
        if not t or t.startswith("."):
            if re.match(r"^\.LBB\S*:", t) or re.match(r"^_Z\S*:", t):
                insts.append((n, "LABEL"))
            continue
        insts.append((n, t))
    for i, (n, t) in enumerate(insts):
        op, ops = operands(t)
        if "_dpp" not in op or t == "LABEL" or len(ops) < 2:
            continue
        src = regs(ops[1].split()[0])
        waits = 0
        j = i - 1
        while j >= 0 and waits < 2:
            pn, pt = insts[j]
            if pt == "LABEL":
                break
            pop, pops = operands(pt)
            if pop == "s_nop":
                waits += int(pops[0], 0) + 1
            else:
                if pop.startswith("v_") and not pop.startswith("v_cmp") and pops:
                    if regs(pops[0].split()[0]) & src:
                        bad.append((n + 1, t, pn + 1, pt, waits))
                        break
                waits += 1
            j -= 1
    return bad


def main():
    lines = open(sys.argv[1]).read().split("\n")
    bad = check(lines)
    for n, t, pn, pt, w in bad:
        print(f"line {n}: {t}\n   <- line {pn} ({w} wait states): {pt}")
    print(f"{len(bad)} DPP hazards")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
