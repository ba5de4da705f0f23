#!/usr/bin/env python3
"""Benchmark: Newton steps/sec + factor TFLOP/s on the dense QP n=8192
(BASELINE.json configs[2], "C3": n=8192, m=2048 inequality rows, p=1024
equality rows -> KKT N = 11264, augmented LDL^T), synthetic data (SURVEY.md
§8d generator, seed 1234 + rank), generated in place in HBM.

A "step" is one Newton iteration of Optimizer::solve_quasi_definite_
(Optimizer.cpp:127-219) on the device: KKT assembly, blocked LDL^T, two
(rhs + triangular solves + back-substitution), two ratio tests, mu_aff/sigma,
update, and the next iterate's residuals/objective/mu.  A converged iterate
is reset to the initial point on the device (no host round trip), so every
timed step is a full Newton step.

Multi-GPU (torchrun, one process per GPU): each rank solves its own
independent QP -- the path does not shard a single QP (replicas, weak
scaling) -- and RCCL all-reduces only the convergence scalars
(max res, max mu, sum converged) once per step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X dense fp64 matrix peak (BASELINE.md "Peaks")

WORKLOADS = {
    "c3": dict(n=8192, m=2048, p=1024, sample_scale=2, desc="dense QP n=8192, m=2048 ineq (SlackedSlacks), p=1024 eq "
                                          "(Regularization), augmented LDL^T, KKT N=11264"),
    "c2": dict(n=2048, m=512, p=0, normal=True, sample_scale=1,
               desc="dense QP n=2048, m=512 ineq, normal equations: Cholesky(H) + TRSM + SYRK + Cholesky(S)"),
    "c2_aug": dict(n=2048, m=512, p=0, sample_scale=1, desc="C2's QP (n=2048, m=512) with the augmented LDL^T, for comparison"),
    "small": dict(n=1024, m=256, p=128, desc="dense QP n=1024, m=256, p=128 (smoke size)"),
    "c5": dict(n=16384, m=0, p=0, mixed=True, sample_scale=8,
               desc="dense QP n=16384 box-only (SlackedSlacks), fp32 LDL^T of the scaled KKT + fp64 iterative "
                    "refinement to 1e-12"),
    "c4": dict(n=256, m=64, p=0, batch=1024, sample_scale=1,
               desc="batch of 1024 independent dense QPs n=256, m=64 ineq (KKT N=320), sharded across ranks; "
                    "one launch per phase for a rank's whole shard"),
    "c5_f64": dict(n=16384, m=0, p=0, sample_scale=8,
                   desc="C5's QP (n=16384 box-only) with the plain fp64 factor, for comparison"),
}
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X f32-input MFMA peak (MI355X_MICROARCH.md, Matrix cores)


def cpu_baseline(wl):
    """Time the CPU oracle (a bit-faithful restatement of the reference path,
    oracle/ipmz_oracle.cpp, single thread) on a bounded sample: one Newton
    step of the same workload with every dimension divided by sample_scale,
    extrapolated per phase by its complexity (LDL^T N^3, assembly and the
    rest O(N^2)).  The reference itself cannot run C3 (its evaluator asserts on
    the Regularization block, Evaluation.cpp:57-60)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test/baseline infrastructure only

    sample_scale = wl.get("sample_scale", 4)
    n, m, p = (wl[k] // sample_scale for k in ("n", "m", "p"))
    if wl.get("batch"):  # C4: QP-steps/s of one core, from a bounded run of whole QPs
        steps = 0
        seed = 0
        wall = 0.0
        while wall < 10.0:
            o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed))  # generation is not timed
            t1 = time.perf_counter()
            for _ in range(3):
                o.iterate()
                steps += 1
            wall += time.perf_counter() - t1
            seed += 1
        return {"value": steps / wall, "unit": "QP-steps/s", "cores": 1, "kind": "port",
                "sample": f"{steps} Newton steps of the oracle on {seed} QPs n={n}, m={m} (3 steps each) in "
                          f"{wall:.1f} s, single thread; cpu={platform.processor() or platform.machine()}"}
    qp = oracle.gen_qp(n, m, p, 1234)
    o = oracle.OracleQP(qp)
    t0 = time.perf_counter()
    _, _, ph = o.iterate_timed()
    wall = time.perf_counter() - t0
    Ns = n + m + p
    Nf = wl["n"] + wl["m"] + wl["p"]
    r = Nf / Ns
    head = wall - (ph["assemble"] + ph["ldlt"] + ph["rest"])  # objective/res/mu evaluation
    t_full = ph["ldlt"] * r ** 3 + (ph["assemble"] + ph["rest"] + head) * r ** 2
    return {
        "value": 1.0 / t_full,
        "unit": "steps/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"1 Newton step of the oracle at n={n}, m={m}, p={p} (N={Ns}) took {wall:.2f} s "
                   f"(LDL^T {ph['ldlt']:.2f} s); extrapolated to N={Nf} as LDL^T x{r ** 3:.0f} (N^3) + "
                   f"rest x{r ** 2:.0f} (N^2) = {t_full:.1f} s/step; cpu={platform.processor() or platform.machine()}"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--nbo", type=int, default=int(os.environ.get("IPMZ_NBO", 0)),
                    help="outer panel width; 0 = libipmz's choice by matrix order (384 for N >= 8192, else 256)")
    ap.add_argument("--nbi", type=int, default=int(os.environ.get("IPMZ_NBI", 64)))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ir-tol", type=float, default=1e-12, help="c5: refinement tolerance")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events (allows graph replay)")
    ap.add_argument("--batch", type=int, default=0, help="c4: override the global batch (e.g. 128 = one rank's "
                                                          "shard at 8 GPUs, measured on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # IPMZ_BENCH_SHARED_DEVICE=1: every rank on cuda:0 with the gloo backend --
    # a rehearsal of the multi-rank path on a one-GPU box (not a measurement)
    shared = os.environ.get("IPMZ_BENCH_SHARED_DEVICE") == "1"
    if shared:
        local_rank = 0
    if world > 1:
        torch.cuda.set_device(local_rank)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)

    import ipmz_amd as I

    wl = WORKLOADS[args.workload]
    n, m, p = wl["n"], wl["m"], wl["p"]
    Nk = n + m + p
    stream = torch.cuda.current_stream()
    ctx = I.Context(local_rank, stream=stream.cuda_stream, nbo=args.nbo, nbi=args.nbi)
    nbatch = wl.get("batch", 0)
    if nbatch and args.batch:
        nbatch = args.batch
    if nbatch:  # C4: this rank's contiguous shard of the batch, one Batch object
        from ipmz_amd.dist import shard
        mine = shard(nbatch, world, rank)
        B = len(mine)
        qp = I.Batch(n, m, p, B, ctx)
        qp.generate(mine.start)  # QP i has seed i, as in the single-GPU batch
    else:
        B = 1
        qp = I.Optimizer(n, m, p, ctx)
        qp.generate(1234 + rank)
    mixed = wl.get("mixed", False)
    if mixed:
        qp.set_mixed_precision(True, args.ir_tol, 20)
    if wl.get("normal"):
        qp.set_reduction(I.REDUCTION_NORMAL)
    timing = not args.no_timing
    flags = I.STEP_RESTART_IF_CONVERGED | (0 if timing else I.STEP_GRAPH)
    from ipmz_amd.dist import pack_summary, reduce_summary

    sc = torch.zeros(B, I.SC_COUNT, dtype=torch.float64, device="cuda")

    def one_step():
        qp.step(flags)
        if world > 1:
            # RCCL all-reduce of the convergence summary only,
            # enqueued on the solver's stream: no host round trip
            if nbatch:
                qp.copy_batch_scalars(sc.data_ptr())
            else:
                qp.copy_scalars(sc.data_ptr())
            reduce_summary(pack_summary(sc[:, I.SC["res"]].max(), sc[:, I.SC["mu"]].max(),
                                        sc[:, I.SC["converged"]].sum(), "cuda"))

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if timing:
        qp.set_timing(True)  # resets the phase accumulators
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    s = qp.scalars()
    ph = qp.phase_times() if timing else None

    if rank == 0:
        steps_total = args.steps * (nbatch if nbatch else world)
        value = steps_total / elapsed
        out = {
            "metric": (f"QP Newton steps/sec, batch of {nbatch} dense QPs n=256, 1/2/4/8 MI355X" if nbatch else
                       "Newton steps/sec + factor TFLOP/s, dense QP n=8192, 1/2/4/8 MI355X"),
            "value": value,
            "unit": "QP-steps/s" if nbatch else "steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if nbatch else "weak",
            "vs_baseline": None,
            "dtype": "f32 factor + f64 refinement" if mixed else "f64",
            "data": "synthetic (SURVEY.md §8d splitmix64 generator, generated in HBM; seed 1234+rank)",
            "config": {"workload": args.workload, "n": n, "m": m, "p": p, "kkt_N": Nk,
                       "formulation": ("SlackedSlacks box-only, fp32 LDL^T of S K S + fp64 iterative refinement "
                                       f"(tol {args.ir_tol:g})") if mixed else
                                      ("SlackedSlacks" + (" ineq" if m else " box-only") +
                                       (" + Regularization eq (delta=1e-4)" if p else "") +
                                       (", normal equations (Cholesky H, S)" if wl.get("normal") else
                                        ", augmented LDL^T")),
                       "parallelism": (f"batch sharded over {world} rank(s), {B} QPs on rank 0" if nbatch else
                                       f"replicas x{world} (independent QPs)") +
                                      ", RCCL all-reduce of the convergence summary only",
                       "blocking": {"nbo": args.nbo or (384 if Nk >= 8192 and args.nbi == 64 else 256),
                                    "nbi": args.nbi},
                       "description": wl["desc"]},
            "restarts": s["restarts"],
        }
        traffic = None
        tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(tpath) and args.workload == "c3":  # HBM bytes per trailing launch, committed PMC passes of C3
            with open(tpath) as f:
                traffic = json.load(f)
            traffic["source"] = os.path.relpath(tpath, REPO) + " (" + traffic.get("profile", "") + ")"
        if ph:
            k = args.steps
            factor_ms = ph["factor"] / k
            out["factor_tflops"] = B * (Nk ** 3 / 3.0) / (factor_ms * 1e-3) / 1e12
            out["phase_ms_per_step"] = {kk: ph[kk] / k for kk in ("step", "assemble", "factor", "solve", "eval")}
            tr_s = ph["trailing"] * 1e-3
            launches = ph["trailing_launches"]
            achieved = ph["trailing_flops"] / tr_s / 1e12 if tr_s > 0 else 0.0
            peak = FP32_MFMA_PEAK_TFLOPS if mixed else FP64_MFMA_PEAK_TFLOPS
        if ph and not nbatch and ph["trailing_launches"] == 0:
            # no trailing update reaches the 128 x 128 kernel (C2: orders 2048
            # and 512): the whole factor phase against the fp64 MFMA peak
            if wl.get("normal"):
                fl = n ** 3 / 3.0 + n * n * (m + p) + n * (m + p) ** 2 + (m + p) ** 3 / 3.0
                what = "normal-equations factor phase: LDL^T(H) + TRSM + SYRK + LDL^T(S)"
            else:
                fl = Nk ** 3 / 3.0
                what = "LDL^T factor phase"
            ach = fl / (factor_ms * 1e-3) / 1e12
            out["roofline"] = {"bound": "mfma", "kernel": what, "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                               "frac": ach / peak, "traffic": None,
                               "note": "algorithmic flops over the factor phase time (HIP events)"}
        elif ph and nbatch:
            # batched factor: every launch serves the whole shard; the bound at
            # N = 320 is latency, priced here against the fp64 MFMA peak
            out["roofline"] = {"bound": "mfma", "kernel": "ldlt_small_kernel (whole LDL^T of each QP in one 8-wave workgroup, fp64 MFMA)",
                               "achieved": out["factor_tflops"], "peak": peak, "unit": "TFLOP/s",
                               "frac": out["factor_tflops"] / peak, "traffic": None,
                               "note": "factor flops B*N^3/3 over the factor phase time (HIP events)"}
        elif ph:
            out["roofline"] = {
                "bound": "mfma",
                "kernel": (f"gemm_nt_kernel<{'float' if mixed else 'double'},128,128,EPI_SUB,"
                           f"{'2,4' if mixed else '4,4'}> (trailing update A22 -= W21 L21^T, "
                           f"{'fp32' if mixed else 'fp64'} MFMA)"),
                "achieved": achieved,
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": achieved / peak,
                "traffic": traffic.get("traffic_bytes_per_launch") if traffic else None,
                "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes)",
                "traffic_source": traffic.get("source") if traffic else None,
                "algorithmic_bytes_per_launch": traffic.get("algorithmic_bytes_per_launch") if traffic else None,
                "launches": launches,
                "avg_launch_ms": ph["trailing"] / max(1, launches),
                "flops_per_launch": ph["trailing_flops"] / max(1, launches),
            }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(wl)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
