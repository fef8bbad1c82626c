"""Static issue-slot count per IPM phase of one kernel in a listing built with -DOSC_PHASE_MARKS
(the STAMP_BEGIN / STAMP_END points become ';@@' labels).  Diagnostic only: a wavefront alone on
its SIMD pays ~4.5 clocks per issue slot (tools/mb/mb_issue.hip), s_nop N taking N + 1.

    python tools/phase_slots.py file.s [kernel-substring]"""
import re
import sys
from collections import Counter, defaultdict

NAMES = ["stage+rows", "iter-head", "contact blocks", "LDL^T", "rhs", "solve", "Gdy+ratio+reduce",
         "update", "rd", "rank-1 U", "refine: K_A+LDL", "refine: steps"]


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "ELb1ELb0ELi2EE"
    lines = open(path).read().split("\n")
    i0 = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l) and key in l.split(":")[0])
    i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
    slots, mix = Counter(), defaultdict(Counter)
    cur = None
    for l in lines[i0:i1]:
        t = l.strip()
        if ";@@BEGIN" in t:
            cur = "open"
            continue
        m = re.search(r";@@END (\d+)", t)
        if m:
            # attribute the instructions since the last BEGIN to this slot
            for op, n in mix["open"].items():
                mix[int(m.group(1))][op] += n
            slots[int(m.group(1))] += slots["open"]
            slots["open"] = 0
            mix["open"] = Counter()
            cur = None
            continue
        if cur is None or not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        n = int(t.split()[1].rstrip(","), 0) + 1 if op == "s_nop" else 1
        slots["open"] += n
        mix["open"][op] += n
    tot = sum(v for k, v in slots.items() if k != "open")
    for k in sorted(k for k in slots if k != "open"):
        top = ", ".join(f"{o} {n}" for o, n in mix[k].most_common(6))
        print(f"{k:2d} {NAMES[k]:18s} {slots[k]:6d}  {top}")
    print("total", tot)


if __name__ == "__main__":
    main()
