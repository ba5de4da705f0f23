#!/usr/bin/env python3
"""HBM traffic per launch of the trailing-update GEMM from two rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --steps 1 --warmup 0`.

Corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE/WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports half the bytes of a 16-B/lane streaming read,
so it is doubled.  Writes are counted as is.  The counters are memory-side
(L2 -> fabric) requests, so Infinity-Cache hits are included.

Algorithmic bytes of one trailing launch (rank-nbo update of an R x R lower
triangle): C read + written once, W and L panels read once:
    16 * R (R + 1) / 2 + 2 * 8 * R * nbo
R per launch is recovered from the grid size (triangular grid of 128 x 128
tiles; grid / workgroup size).

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write <profile label> > profiles/pmc_traffic.json
    IPMZ_PMC_PREC=32 python tools/pmc_traffic.py ... > profiles/pmc_traffic_c5.json   (C5's fp32 trailing update)
(IPMZ_PMC_NBO: the outer panel width of the profiled run, default 512 = C3's and C5's)
"""
import csv
import json
import math
import sys

import os

PREC = int(os.environ.get("IPMZ_PMC_PREC", 64))
KERNEL = ("dgemm_nt_glds_kernel<128, 128, 4, 4, 8, 3, 8, 0>" if PREC == 64  # C3's trailing update (gemm64.h)
          else "sgemm_nt_glds_kernel<128, 128, 2, 2, 16, 3, 2, 0, true>")   # C5's (gemm32.h)
ES = PREC // 8  # bytes per element
NBO = int(os.environ.get("IPMZ_PMC_NBO", 512))  # the bench's outer panel width (C3, C5: 512)


def rows(d):
    out = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        out.setdefault(r["Kernel_Name"], []).append(r)
    return out


def main():
    f, w = rows(sys.argv[1]), rows(sys.argv[2])
    name = next(k for k in f if KERNEL in k)
    fr, wr = f[name], w[name]
    assert len(fr) == len(wr)
    tot_f = tot_w = tot_alg = 0.0
    for a, b in zip(fr, wr):
        wgs = int(a["Grid_Size"]) // int(a["Workgroup_Size"])
        t = int((math.isqrt(8 * wgs + 1) - 1) // 2)  # tiles per side
        R = t * 128  # tile-rounded trailing order (upper bound of R)
        tot_f += 2.0 * float(a["Counter_Value"]) * 1024
        tot_w += float(b["Counter_Value"]) * 1024
        tot_alg += 2.0 * ES * R * (R + 1) / 2 + 2.0 * ES * R * NBO
    n = len(fr)
    per = (tot_f + tot_w) / n
    out = {
        "kernel": name.split("(")[0],
        "launches": n,
        "fetch_bytes_per_launch": tot_f / n,
        "write_bytes_per_launch": tot_w / n,
        "traffic_bytes_per_launch": per,
        "algorithmic_bytes_per_launch": tot_alg / n,
        "traffic_over_algorithmic": per / (tot_alg / n),
        "profile": sys.argv[3] if len(sys.argv) > 3 else "",
        "nbo": NBO,
        "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB->B; one bench.py step, "
                "separate --pmc passes; algorithmic = C lower triangle read+write + W, L panels",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
