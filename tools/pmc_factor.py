#!/usr/bin/env python3
"""Per-step HBM traffic and MFMA counters of the factorization phase, from
separate rocprofv3 --pmc passes of ONE bench step
(`bench.py --steps 1 --warmup 0 --no-instrumented --no-batched --no-configs
--no-cpu-baseline`, see tools/gpu_round.sh steps pmcf_*):

    pass fetch : FETCH_SIZE
    pass write : WRITE_SIZE
    pass mops  : SQ_INSTS_VALU_MFMA_MOPS_F64
    pass busy  : SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES

The factor phase = every launch of the factor's kernels (trailing / strip
GEMMs, the panel chain and rows launches, the solve prep).  Corrections
(MI355X_MICROARCH.md, HBM / PMC): FETCH_SIZE and WRITE_SIZE are KiB,
FETCH_SIZE reports half the bytes of a 16-B/lane read on gfx950 (doubled);
SQ_INSTS_VALU_MFMA_MOPS_F64 / _F32 count 512-flop units (C5's fp32 factor:
the _F32 counter in the mops pass, PMCW=c5 in tools/gpu_round.sh).

    python tools/pmc_factor.py <fetch dir> <write dir> <mfma dir[,dir...]> <label> <N> [B] > profiles/factor_traffic_c3.json

(the MFMA counters may come from several smaller passes, comma-separated:
one large pass slows every dispatch enough that the panel path's cross-launch
hand-offs can hit their spin limit under the profiler's serialization)
"""
import csv
import json
import sys
from collections import defaultdict

FACTOR_KERNELS = ("gemm_nt_kernel", "gemm_nt_glds_kernel", "panel_kernel", "panel_chain_kernel", "panel_rows_kernel", "solve_prep_kernel",
                  "ldlt_small_kernel", "ldlt_small_pair_kernel", "ldlt_small_ws_kernel", "ldlt_small_left_kernel",  # (the small.hip kernels: C4's batched factor)
                  )


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # kernel -> counter -> sum over launches
    launches = defaultdict(set)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0]
        if not any(k in name for k in FACTOR_KERNELS):
            continue
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    return per, {k: len(v) for k, v in launches.items()}


def main():
    fetch, nf = load(sys.argv[1])
    write, _ = load(sys.argv[2])
    mfma = defaultdict(lambda: defaultdict(float))
    for d in sys.argv[3].split(","):
        part, _ = load(d)
        for k, cs in part.items():
            for c, v in cs.items():
                mfma[k][c] += v
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    N = int(sys.argv[5]) if len(sys.argv) > 5 else 11264
    B = int(sys.argv[6]) if len(sys.argv) > 6 else 1  # QPs per factor phase (C4: 1024)
    kernels = sorted(set(fetch) | set(write) | set(mfma))
    rows = {}
    tot = defaultdict(float)
    for k in kernels:
        fb = 2.0 * fetch[k].get("FETCH_SIZE", 0.0) * 1024
        wb = write[k].get("WRITE_SIZE", 0.0) * 1024
        mops = mfma[k].get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
        mops32 = mfma[k].get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)
        row = {"launches": nf.get(k, 0), "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
               "f64_mfma_flops": 512.0 * mops, "f32_mfma_flops": 512.0 * mops32,
               "mfma_busy_cycles": mfma[k].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0),
               "grbm_gui_active": mfma[k].get("GRBM_GUI_ACTIVE", 0.0),
               "busy_cu_cycles": mfma[k].get("SQ_BUSY_CU_CYCLES", 0.0)}
        rows[k] = row
        for f in ("fetch_bytes", "write_bytes", "hbm_bytes", "f64_mfma_flops", "f32_mfma_flops", "mfma_busy_cycles",
                  "busy_cu_cycles"):
            tot[f] += row[f]
    alg_flops = B * N ** 3 / 3.0
    out = {
        "profile": label,
        "N": N,
        "batch": B,
        "factor_traffic_bytes_per_step": tot["hbm_bytes"],
        "mfma": {
            "f64_mfma_flops_per_step": tot["f64_mfma_flops"],
            "f32_mfma_flops_per_step": tot["f32_mfma_flops"],
            "algorithmic_flops_per_step": alg_flops,
            "executed_over_algorithmic": ((tot["f64_mfma_flops"] + tot["f32_mfma_flops"]) / alg_flops
                                          if alg_flops else None),
            "mfma_busy_cycles": tot["mfma_busy_cycles"],
            "busy_cu_cycles": tot["busy_cu_cycles"],
            "mfma_busy_over_busy_cu": (tot["mfma_busy_cycles"] / tot["busy_cu_cycles"]
                                       if tot["busy_cu_cycles"] else None),
            # the MFMA-busy counter counts per SIMD (4 per CU): the utilisation
            # of the matrix pipes while the CUs are busy, <= 1
            "mfma_util_per_simd": (tot["mfma_busy_cycles"] / (4.0 * tot["busy_cu_cycles"])
                                   if tot["busy_cu_cycles"] else None),
        },
        "per_kernel": rows,
        "note": "one bench step (one factorization), separate --pmc passes, counters summed over the factor's "
                "launches; FETCH_SIZE x2 + WRITE_SIZE (KiB -> B); MFMA flops = 512 x SQ_INSTS_VALU_MFMA_MOPS_F64 "
                "(executed, incl. the masked upper halves of diagonal tiles); mfma_busy_over_busy_cu = "
                "SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CU_CYCLES as reported (both summed over the chip; the MFMA "
                "counter sums the 4 SIMDs of a CU), mfma_util_per_simd = that / 4",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
