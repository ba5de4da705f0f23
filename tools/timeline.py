#!/usr/bin/env python3
"""Print the kernel timeline of the last Newton step in a rocprofv3
--kernel-trace CSV (factor phase analysis): start offset, duration, queue."""
import csv
import sys

rs = list(csv.DictReader(open(sys.argv[1])))
rs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-44:],
             r["Queue_Id"], int(r["Grid_Size_X"])) for r in rs)
i0 = [i for i, r in enumerate(rs) if "k_assemble" in r[2]][-1]
step = rs[i0:]
t0 = step[0][0]
head = int(sys.argv[2]) if len(sys.argv) > 2 else 40
tail = int(sys.argv[3]) if len(sys.argv) > 3 else 40
sel = step if head + tail >= len(step) else step[:head] + [None] + step[-tail:]
for r in sel:
    if r is None:
        print("...")
        continue
    print(f"{(r[0] - t0) / 1e3:9.1f} {(r[1] - r[0]) / 1e3:8.1f} q{r[3]} {r[4]:8d} {r[2]}")
