#!/usr/bin/env python3
"""Critical-path view of the LAST factorization in a rocprofv3 --kernel-trace
CSV (bench.py run): the factor phase is the kernels between the last
k_assemble and the first solve kernel after it.  Prints, per queue, busy time
and idle gaps, and per outer panel the panel launch and what the other queue
ran meanwhile.

    python tools/factor_timeline.py <kernel_trace.csv> [--all] [--at i]   (i-th assembly, default -1 = last)
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for key, s in (("outer_panel", "panel"), ("panel_kernel", "panel"), ("panel_chain", "chain"), ("panel_rows", "rows"), ("0, 4, 4", "trail128"), ("0, 2, 2", "trail64"),
                   ("3, 2, 4", "strip"), ("3, 2, 2", "strip64"), ("3, 4, 4", "strip16w"), ("1, 4, 2", "trsm"),
                   ("panel_trsm", "ptrsm"), ("trsv", "solve"), ("fillBuffer", "memset")):
        if key in n:
            return s
    return n[-30:]


def main():
    path = sys.argv[1]
    rs = []
    for r in csv.DictReader(open(path)):
        rs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?"),
                   int(r.get("Grid_Size_X", r.get("Grid_Size", 0)))))
    rs.sort()
    # bench trace: after the last KKT assembly; kbench trace: after the last fill
    at = int(sys.argv[sys.argv.index("--at") + 1]) if "--at" in sys.argv else -1
    starts = [i for i, r in enumerate(rs) if "k_assemble" in r[2] or "fill_qd" in r[2]]
    print(f"{len(starts)} factor phases in the trace; showing #{at}")
    ia = starts[at]
    fac = []
    for r in rs[ia + 1:]:
        if "trsv" in r[2] or "fill_qd" in r[2]:
            break
        fac.append(r)
    t0 = fac[0][0]
    t1 = max(r[1] for r in fac)
    print(f"factor span {(t1 - t0) / 1e3:.1f} us, {len(fac)} kernels")
    byq = defaultdict(list)
    for r in fac:
        byq[r[3]].append(r)
    for q, lst in byq.items():
        busy = sum(r[1] - r[0] for r in lst)
        kinds = defaultdict(float)
        for r in lst:
            kinds[short(r[2])] += (r[1] - r[0]) / 1e3
        print(f"queue {q}: {len(lst)} kernels, busy {busy / 1e3:.1f} us; " +
              ", ".join(f"{k} {v:.0f}" for k, v in sorted(kinds.items(), key=lambda x: -x[1])))
    # per-kind totals
    kinds = defaultdict(lambda: [0, 0.0])
    for r in fac:
        k = kinds[short(r[2])]
        k[0] += 1
        k[1] += (r[1] - r[0]) / 1e3
    print("kind totals: " + ", ".join(f"{k} x{v[0]} {v[1]:.0f} us" for k, v in sorted(kinds.items(), key=lambda x: -x[1][1])))
    # union of busy time: the factor's idle time
    ev = sorted([(r[0], 1) for r in fac] + [(r[1], -1) for r in fac])
    depth, last, idle, both = 0, t0, 0, 0
    for t, d in ev:
        if depth == 0:
            idle += t - last
        elif depth >= 2:
            both += t - last
        depth += d
        last = t
    print(f"no kernel running: {idle / 1e3:.1f} us; >= 2 kernels: {both / 1e3:.1f} us")
    if "--all" in sys.argv:
        for r in fac:
            print(f"{(r[0] - t0) / 1e3:9.1f} {(r[1] - r[0]) / 1e3:8.1f} q{r[3]} {r[4]:8d} {short(r[2])}")
        return
    panels = [r for r in fac if "outer_panel" in r[2] or "panel_kernel" in r[2] or "panel_chain" in r[2] or "panel_rows" in r[2]]
    print(f"{'start':>8} {'dur':>7} {'gap':>6}  concurrent (other queue)")
    prev_end = t0
    for p in panels:
        conc = [r for r in fac if r[3] != p[3] and r[0] < p[1] and r[1] > p[0]]
        desc = " ".join(f"{short(r[2])}:{(min(r[1], p[1]) - max(r[0], p[0])) / 1e3:.0f}" for r in conc)
        print(f"{(p[0] - t0) / 1e3:8.1f} {(p[1] - p[0]) / 1e3:7.1f} {(p[0] - prev_end) / 1e3:6.1f}  {desc}")
        prev_end = p[1]


if __name__ == "__main__":
    main()
