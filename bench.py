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
timed step is a full Newton step.  The timed steps run the production path:
HIP-graph replay for steps whose factor does not fork (C4's batches), eager
launches with at most one step in flight for the look-ahead factor (C3, C2,
C5) -- each line's config.timing says which; a second, instrumented pass with
per-phase HIP events gives the phase split and the roofline numbers.

Multi-GPU (torchrun, one process per GPU):
  * headline (C3): each rank solves its own independent QP -- the path does
    not shard a single QP (replicas, weak scaling);
  * "batched" sub-object (C4, BASELINE.json configs[3]): the 1024-QP batch
    (n=256, m=64) sharded over the ranks, strong scaling, with ONE all-reduce
    (MAX) of the device-computed convergence summary per step -- the only
    collective;
  * "batched_shard" sub-object (one GPU only): C4 at 128 QPs, the shard one
    rank holds in the 8-GPU job, measured alone;
  * "configs" sub-object (default c3 run): C2 (normal equations, n=2048) and
    C5 (n=16384, fp32 factor + fp64 refinement), replicas like the headline,
    each with its own roofline and CPU baseline (--no-configs skips them).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5|...]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix peak (BASELINE.md "Peaks")
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X f32-input MFMA peak (MI355X_MICROARCH.md, Matrix cores)

HEADLINE_METRIC = "Newton steps/sec + factor TFLOP/s, dense QP n=8192, 1/2/4/8 MI355X"  # BASELINE.json metric
WORKLOADS = {
    "c3": dict(n=8192, m=2048, p=1024, sample_scale=1, desc="dense QP n=8192, m=2048 ineq (SlackedSlacks), p=1024 eq "
                                          "(Regularization), augmented LDL^T, KKT N=11264"),
    "c2": dict(n=2048, m=512, p=0, normal=True, sample_scale=1,
               desc="dense QP n=2048, m=512 ineq, normal equations: Cholesky(H) + TRSM + SYRK + Cholesky(S)"),
    "c2_aug": dict(n=2048, m=512, p=0, sample_scale=1, desc="C2's QP (n=2048, m=512) with the augmented LDL^T, for comparison"),
    "small": dict(n=1024, m=256, p=128, sample_scale=1, desc="dense QP n=1024, m=256, p=128 (smoke size)"),
    "c5": dict(n=16384, m=0, p=0, mixed=True, sample_scale=2,
               desc="dense QP n=16384 box-only (SlackedSlacks), fp32 LDL^T of the scaled KKT + fp64 iterative "
                    "refinement to 1e-12"),
    "c4": dict(n=256, m=64, p=0, batch=1024, sample_scale=1,
               desc="batch of 1024 independent dense QPs n=256, m=64 ineq (KKT N=320), sharded across ranks; "
                    "one launch per phase for a rank's whole shard"),
    "c5_f64": dict(n=16384, m=0, p=0, sample_scale=8,
                   desc="C5's QP (n=16384 box-only) with the plain fp64 factor, for comparison"),
}


def cpu_start(*args):
    """oracle/cpu_bench.py as a child process (it never touches the GPU)."""
    return subprocess.Popen([sys.executable, os.path.join(REPO, "oracle", "cpu_bench.py"), *map(str, args)],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def cpu_finish(proc, name=""):
    t0 = time.perf_counter()
    while True:  # a progress line on stderr every 30 s (stdout carries only the JSON line)
        try:
            out, err = proc.communicate(timeout=30)
            break
        except subprocess.TimeoutExpired:
            el = time.perf_counter() - t0
            if el > 900:
                proc.kill()
                proc.communicate()
                return {"error": "timed out after 900 s"}
            print(f"[bench] CPU baseline {name}: running ({el:.0f} s)", file=sys.stderr, flush=True)
    if proc.returncode != 0:
        return {"error": err[-400:]}
    return json.loads(out.strip().splitlines()[-1])


def cpu_baselines(names):
    """The single-core CPU legs of `names` side by side, each pinned to its own
    core (so the wall time is the longest one, ~3 min for a full-size C3
    step), then C4's all-core leg alone (it takes 16 cores)."""
    procs, slot = {}, 0
    for w in names:
        wl = WORKLOADS[w]
        if wl.get("batch"):
            procs[w] = cpu_start("batch", wl["n"], wl["m"], 10, 1, slot)  # its own core, like the step legs
        else:
            procs[w] = cpu_start("step", wl["n"], wl["m"], wl["p"], wl.get("sample_scale", 4), slot)
        slot += 1
    print(f"[bench] CPU baselines {', '.join(names)} on the host cores (a full-size C3 step takes ~3 min)",
          file=sys.stderr, flush=True)
    out = {w: cpu_finish(p, w) for w, p in procs.items()}
    for w in names:
        wl = WORKLOADS[w]
        if wl.get("batch"):
            out[w]["all_cores"] = cpu_finish(cpu_start("batch", wl["n"], wl["m"], 8, 16), w + " (16 cores)")
    return out


def load_json(rel):
    path = os.path.join(REPO, rel)
    if not rel or not os.path.isfile(path):
        return None
    with open(path) as fh:
        out = json.load(fh)
    out["source"] = rel
    return out


def timed(world, dist, torch, steps, fn):
    """Barrier + sync on both sides of exactly `steps` calls; max over ranks."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    return elapsed


def run_batched(I, ctx, args, world, rank, dist, torch, wl, nbatch):
    """C4: this rank's contiguous shard of the batch as one Batch; per step
    one device summary kernel + ONE all-reduce (MAX) on the solver's stream."""
    from ipmz_amd.dist import reduce_summary, shard
    mine = shard(nbatch, world, rank)
    B = len(mine)
    qp = I.Batch(wl["n"], wl["m"], wl["p"], B, ctx)
    qp.generate(mine.start)  # QP i has seed i, as in the single-GPU batch
    buf = torch.zeros(3, dtype=torch.float64, device="cuda")
    flags = I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH

    def one_step(f=flags):
        qp.step(f)
        qp.summary_into(buf)
        reduce_summary(buf)

    for _ in range(args.warmup):
        one_step()
    elapsed = timed(world, dist, torch, args.steps, one_step)
    graph = qp.last_step_graph()
    # instrumented pass (per-phase HIP events, eager launches)
    N = wl["n"] + wl["m"] + wl["p"]
    ph, fac = None, None
    if not args.no_instrumented:
        qp.set_timing(True)
        for _ in range(args.steps):
            one_step(I.STEP_RESTART_IF_CONVERGED)
        torch.cuda.synchronize()
        ph = qp.phase_times()
        factor_ms = ph["factor"] / args.steps
        fac = B * (N ** 3 / 3.0) / (factor_ms * 1e-3) / 1e12
    out = {
        "metric": f"QP Newton steps/sec, batch of {nbatch} dense QPs n={wl['n']} (C4), 1/2/4/8 MI355X",
        "value": args.steps * nbatch / elapsed, "unit": "QP-steps/s", "n_gpus": world,
        "ms_per_step": 1e3 * elapsed / args.steps, "scaling": "strong", "higher_is_better": True,
        "config": {"workload": "c4", "n": wl["n"], "m": wl["m"], "kkt_N": N, "global_batch": nbatch,
                   "qps_on_rank0": B, "parallelism": f"batch sharded over {world} rank(s); one all-reduce (MAX) "
                                                     "of {max res, max mu, unconverged} per step",
                   "timing": ("HIP-graph replay" if graph else "eager launches") + " of the whole step + the "
                             "summary kernel + the all-reduce; phases from a second, instrumented pass"},
        "phase_ms_per_step": ({k: ph[k] / args.steps for k in ("step", "assemble", "factor", "solve", "eval")}
                              if ph else None),
        "roofline": {"bound": "mfma", "kernel": "batched factor phase (whole left-looking LDL^T of each QP in "
                                                "one 8-wave workgroup: diagonal chain on waves 0-3, tiles on "
                                                "4-7; fp64 MFMA)",
                     "achieved": fac, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": fac / FP64_MFMA_PEAK_TFLOPS if fac else None, "traffic": None,
                     "note": "B * N^3/3 over the factor phase (HIP events), rank 0"},
    }
    ftr = load_json("profiles/factor_traffic_c4.json") if nbatch == 1024 and world == 1 else None
    if ftr:
        out["roofline"]["traffic"] = ftr.get("factor_traffic_bytes_per_step")
        out["roofline"]["traffic_source"] = ftr["source"]
        out["roofline"]["mfma"] = ftr.get("mfma")
    qp.close()
    return out


def shard_line(I, ctx, args, dist, torch):
    """C4 at one rank's shard of the 8-GPU job (1024 / 8 = 128 QPs), on this
    one GPU: the per-GPU regime an 8-GPU run times (128 workgroups on 256
    CUs, the 16-wave solve), graph-replayed like the 1024-QP line."""
    sub = run_batched(I, ctx, args, 1, 0, dist, torch, WORKLOADS["c4"], 128)
    sub["metric"] = "QP Newton steps/sec, one rank's C4 shard (128 of 1024 QPs, n=256) on one MI355X"
    sub["config"]["note"] = ("the shard each rank holds when the 1024-QP batch runs on 8 GPUs, measured alone "
                             "(no collective); 8 x this value bounds the 8-GPU C4 line")
    return sub


def run_single(I, ctx, args, world, dist, torch, workload):
    """One QP per rank (replicas): the timed HIP-graph pass, then the
    instrumented pass for the phase split and the roofline."""
    wl = WORKLOADS[workload]
    n, m, p = wl["n"], wl["m"], wl["p"]
    Nk = n + m + p
    mixed = wl.get("mixed", False)
    peak = FP32_MFMA_PEAK_TFLOPS if mixed else FP64_MFMA_PEAK_TFLOPS
    rank = dist.get_rank() if world > 1 else 0
    qp = I.Optimizer(n, m, p, ctx)
    qp.generate(1234 + rank)
    if mixed:
        qp.set_mixed_precision(True, args.ir_tol, 20)
    if wl.get("normal"):
        qp.set_reduction(I.REDUCTION_NORMAL)
    flags = I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH
    for _ in range(args.warmup):
        qp.step(flags)
    elapsed = timed(world, dist, torch, args.steps, lambda: qp.step(flags))
    graph = qp.last_step_graph()
    ph = None
    if not args.no_instrumented:
        qp.set_timing(True)  # resets the phase accumulators; eager launches with HIP events
        t_ins = timed(world, dist, torch, args.steps, lambda: qp.step(I.STEP_RESTART_IF_CONVERGED))
        ph = qp.phase_times()
    s = qp.scalars()
    out = {
        "metric": (HEADLINE_METRIC if workload == "c3" else
                   f"Newton steps/sec + factor TFLOP/s, {workload.upper()}: {wl['desc']}"),
        "value": args.steps * world / elapsed,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 factor + f64 refinement" if mixed else "f64",
        "data": "synthetic (SURVEY.md §8d splitmix64 generator, generated in HBM; seed 1234+rank)",
        "config": {"workload": workload, "n": n, "m": m, "p": p, "kkt_N": Nk,
                   "formulation": ("SlackedSlacks box-only, fp32 LDL^T of S K S + fp64 iterative refinement "
                                   f"(tol {args.ir_tol:g})") if mixed else
                                  ("SlackedSlacks" + (" ineq" if m else " box-only") +
                                   (" + Regularization eq (delta=1e-4)" if p else "") +
                                   (", normal equations (Cholesky H, S)" if wl.get("normal") else
                                    ", augmented LDL^T")),
                   "parallelism": f"replicas x{world} (independent QPs, one per GPU)",
                   "blocking": dict(zip(("nbo", "nbi"), ctx.blocking(Nk))),
                   "timing": ("HIP-graph replay of the whole step" if graph else
                              "eager launches of the whole step (its factor forks onto the look-ahead streams), "
                              "at most one step in flight") +
                             " (production path); phases from a second, instrumented pass",
                   "description": wl["desc"]},
        "restarts": s["restarts"],
    }
    if mixed:  # refinement corrections of the last step's two solves
        out["ir"] = {"iters_affine": s["ir_iters_aff"], "iters_corrector": s["ir_iters"],
                     "ratio_affine": s["ir_ratio_aff"], "ratio_corrector": s["ir_ratio"]}
    if ph:
        k = args.steps
        factor_ms = ph["factor"] / k
        out["value_instrumented"] = k * world / t_ins
        out["factor_tflops"] = (Nk ** 3 / 3.0) / (factor_ms * 1e-3) / 1e12
        out["phase_ms_per_step"] = {kk: ph[kk] / k for kk in ("step", "assemble", "factor", "solve", "eval")}
        if wl.get("normal"):
            fl = n ** 3 / 3.0 + n * n * (m + p) + n * (m + p) ** 2 + (m + p) ** 3 / 3.0
            what = ("normal-equations factor phase: Cholesky(H) + TRSM + SYRK + Cholesky(S) as one pipelined "
                    "x-first blocked LDL^T (fp64 MFMA)")
        else:
            fl = Nk ** 3 / 3.0
            what = ("blocked LDL^T factor phase (" + ("fp32 " if mixed else "fp64 ") +
                    "MFMA; outer-panel and trailing/strip GEMM launches on two streams)")
        ach = fl / (factor_ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": what, "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                "frac": ach / peak, "traffic": None,
                "note": "algorithmic flops (N^3/3 for LDL^T, SURVEY.md §8d) over the factor phase time "
                        "(HIP events on the solver stream around the phase)"}
        ftr = load_json(f"profiles/factor_traffic_{workload}.json")
        if ftr:
            roof["traffic"] = ftr.get("factor_traffic_bytes_per_step")
            roof["traffic_source"] = ftr["source"]
            roof["mfma"] = ftr.get("mfma")
        tr_s = ph["trailing"] * 1e-3
        launches = ph["trailing_launches"]
        if launches:
            trk = load_json({"c3": "profiles/pmc_traffic.json", "c5": "profiles/pmc_traffic_c5.json"}.get(workload, ""))
            tach = ph["trailing_flops"] / tr_s / 1e12
            roof["trailing"] = {
                "kernel": ("sgemm_nt_kernel<128,128,...> (csrc/gemm32.h, v_mfma_f32_32x32x2_f32; trailing update "
                           "A22 -= W21 L21^T of the fp32 factor, one launch over the lower tiles)" if mixed else
                           "dgemm_nt_glds_kernel<128,128,4,4,8,3> (csrc/gemm64.h, LDS-DMA staging; trailing update "
                           "A22 -= W21 L21^T; gemm_nt_kernel<double,128,128,EPI_SUB,4,4> for launches with partial "
                           "tiles)"),
                "achieved": tach, "peak": peak, "unit": "TFLOP/s", "frac": tach / peak,
                "traffic": trk.get("traffic_bytes_per_launch") if trk else None,
                "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes)",
                "traffic_source": trk.get("source") if trk else None,
                "algorithmic_bytes_per_launch": trk.get("algorithmic_bytes_per_launch") if trk else None,
                "launches": launches, "avg_launch_ms": ph["trailing"] / launches,
                "flops_per_launch": ph["trailing_flops"] / launches,
            }
        out["roofline"] = roof
    qp.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--nbo", type=int, default=int(os.environ.get("IPMZ_NBO", 0)),
                    help="outer panel width; 0 = libipmz's choice by matrix order")
    ap.add_argument("--nbi", type=int, default=int(os.environ.get("IPMZ_NBI", 64)))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-batched", action="store_true", help="skip the C4 'batched' sub-object")
    ap.add_argument("--no-configs", action="store_true", help="c3: skip the C2 / C5 'configs' sub-objects")
    ap.add_argument("--no-instrumented", action="store_true", help="skip the per-phase HIP-event pass")
    ap.add_argument("--ir-tol", type=float, default=1e-12, help="c5: refinement tolerance")
    ap.add_argument("--batch", type=int, default=0, help="c4: override the global batch (e.g. 128 = one rank's "
                                                          "shard at 8 GPUs, measured on one GPU)")
    args = ap.parse_args()

    # the CPU baselines first (rank 0, one GPU): a child process on the host
    # cores while the GPU is idle, so the GPU legs below run back to back
    cpu = {}
    if not args.no_cpu_baseline and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        wl0 = WORKLOADS[args.workload]
        names = [args.workload]
        if not wl0.get("batch") and not args.no_batched:
            names.append("c4")
        if args.workload == "c3" and not args.no_configs:
            names += ["c2", "c5"]
        res = cpu_baselines(names)
        cpu["head"] = res[args.workload]
        if "c4" in res and args.workload != "c4":
            cpu["batched"] = res["c4"]
        cpu.update({w: res[w] for w in ("c2", "c5") if w in res and w != args.workload})

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
    stream = torch.cuda.current_stream()
    ctx = I.Context(local_rank, stream=stream.cuda_stream, nbo=args.nbo, nbi=args.nbi)
    nbatch = wl.get("batch", 0)
    if nbatch and args.batch:
        nbatch = args.batch

    if nbatch:  # C4 as the headline
        head = run_batched(I, ctx, args, world, rank, dist, torch, wl, nbatch)
        out = dict(head)
        if world == 1 and nbatch != 128 and not args.no_batched:
            out["batched_shard"] = shard_line(I, ctx, args, dist, torch)
        out.update({"steps": args.steps, "warmup": args.warmup, "vs_baseline": None, "dtype": "f64",
                    "data": "synthetic (SURVEY.md §8d splitmix64 generator, generated in HBM; QP i: seed i)"})
        out["config"]["description"] = wl["desc"]
        out["config"]["formulation"] = "SlackedSlacks ineq, augmented LDL^T"
    else:
        out = run_single(I, ctx, args, world, dist, torch, args.workload)
        if not args.no_batched:
            out["batched"] = run_batched(I, ctx, args, world, rank, dist, torch, WORKLOADS["c4"], 1024)
            if world == 1:
                out["batched_shard"] = shard_line(I, ctx, args, dist, torch)
        if args.workload == "c3" and not args.no_configs:
            # the other single-GPU configs of BASELINE.json, each its own line item
            out["configs"] = {w: run_single(I, ctx, args, world, dist, torch, w) for w in ("c2", "c5")}
    if rank == 0:
        if cpu:
            out["cpu_baseline"] = cpu["head"]
            if "batched" in out and "batched" in cpu:
                out["batched"]["cpu_baseline"] = cpu["batched"]
            for w, sub in out.get("configs", {}).items():
                if w in cpu:
                    sub["cpu_baseline"] = cpu[w]
        # last key of the line: every config's figures in a few hundred
        # bytes, so a record that keeps only the line's tail still has them
        out["summary"] = summary(out, args.workload)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def summary(out, workload):
    """{config: [value, unit, ms/step, factor ms/step, roofline frac, cpu
    baseline value]} for the headline and every sub-line."""
    def row(d):
        if not d or "value" not in d:
            return None
        ph = d.get("phase_ms_per_step") or {}
        roof = d.get("roofline") or {}
        cpu = (d.get("cpu_baseline") or {}).get("value")

        def r(x, k=4):
            return None if x is None else float(f"{x:.{k}g}")
        return [r(d["value"], 6), d.get("unit"), r(d.get("ms_per_step")), r(ph.get("factor")),
                r(roof.get("frac"), 3), r(cpu)]
    head = out.get("config", {}).get("workload", workload)
    if head == "c4":
        head = f"c4_b{out['config'].get('global_batch')}"
    sm = {"columns": ["value", "unit", "ms_per_step", "factor_ms", "frac", "cpu_value"], head: row(out)}
    if "batched" in out:
        sm[f"c4_b{out['batched']['config']['global_batch']}"] = row(out["batched"])
    if "batched_shard" in out:
        sm["c4_b128"] = row(out["batched_shard"])
    for w, sub in out.get("configs", {}).items():
        sm[w] = row(sub)
    return sm


if __name__ == "__main__":
    main()
