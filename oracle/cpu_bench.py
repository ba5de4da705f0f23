#!/usr/bin/env python3
"""CPU baseline of bench.py: the oracle (a bit-faithful restatement of the
reference's Newton step, oracle/ipmz_oracle.cpp) timed on the host cores.

TEST / BASELINE INFRASTRUCTURE ONLY -- bench.py runs this as a child process
after its timed GPU region (the child never touches the GPU).  The LDL^T is
the reference's own loop order (LinearSolvers.cpp:14-42, serial), not the
blocked form the parity tests use.

    python oracle/cpu_bench.py step  N_n N_m N_p SCALE [SLOT]  one Newton step at dims/SCALE, pinned to one core
                                                          (the SLOT-th available one), extrapolated per phase to
                                                          the full dims (N^3 / N^2); SCALE 1 = measured as is
    python oracle/cpu_bench.py batch n m SECONDS WORKERS [START]  QP-steps/s of WORKERS single-core processes
                                                          (one QP per process at a time, 3 steps each, seeds
                                                          disjoint), worker i pinned to the (START+i)-th
                                                          available core
Prints one JSON object.
"""
import json
import multiprocessing as mp
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def cpu_info():
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    avail = sorted(os.sched_getaffinity(0))
    return model, os.cpu_count(), avail


def pin(cpu):
    os.sched_setaffinity(0, {cpu})
    os.environ["OMP_NUM_THREADS"] = "1"


def step(n, m, p, scale, slot=0):
    model, nproc, avail = cpu_info()
    cpu = avail[slot % len(avail)]
    pin(cpu)
    import oracle
    oracle.set_serial_ldlt(True)  # the reference's loop order
    ns, ms, ps = n // scale, m // scale, p // scale
    o = oracle.OracleQP(oracle.gen_qp(ns, ms, ps, 1234))
    t0 = time.perf_counter()
    _, _, ph = o.iterate_timed()
    wall = time.perf_counter() - t0
    Ns, Nf = ns + ms + ps, n + m + p
    r = Nf / Ns
    head = wall - (ph["assemble"] + ph["ldlt"] + ph["rest"])  # objective / res / mu
    t_full = ph["ldlt"] * r ** 3 + (ph["assemble"] + ph["rest"] + head) * r ** 2
    if scale == 1:
        sample = (f"1 full-size Newton step of the oracle (reference loop order, serial LDL^T) at n={n}, m={m}, "
                  f"p={p} (N={Nf}): {wall:.1f} s (LDL^T {ph['ldlt']:.1f} s), measured, not extrapolated")
    else:
        sample = (f"1 Newton step of the oracle (reference loop order, serial LDL^T) at n={ns}, m={ms}, p={ps} "
                  f"(N={Ns}) took {wall:.2f} s (LDL^T {ph['ldlt']:.2f} s); extrapolated to N={Nf} as "
                  f"LDL^T x{r ** 3:.0f} (N^3) + rest x{r ** 2:.0f} (N^2) = {t_full:.1f} s/step")
    return {"value": 1.0 / t_full, "unit": "steps/s", "cores": 1, "kind": "port", "sample": sample,
            "cpu_model": model, "nproc": nproc, "cpus_available": len(avail), "pinned_cpu": cpu}


def _batch_worker(args):
    cpu, idx, workers, n, m, seconds = args
    pin(cpu)
    import oracle
    oracle.set_serial_ldlt(True)
    steps, wall, seed = 0, 0.0, idx
    while wall < seconds:
        o = oracle.OracleQP(oracle.gen_qp(n, m, 0, seed))  # generation is not timed
        t1 = time.perf_counter()
        for _ in range(3):
            o.iterate()
            steps += 1
        wall += time.perf_counter() - t1
        seed += workers
    return steps, wall


def batch(n, m, seconds, workers, start=0):
    model, nproc, avail = cpu_info()
    workers = max(1, min(workers, len(avail)))
    jobs = [(avail[(start + i) % len(avail)], i, workers, n, m, seconds) for i in range(workers)]
    if workers == 1:
        res = [_batch_worker(jobs[0])]
    else:
        with mp.get_context("fork").Pool(workers) as pool:
            res = pool.map(_batch_worker, jobs)
    steps = sum(s for s, _ in res)
    rate = sum(s / w for s, w in res)  # each worker's own rate, summed
    return {"value": rate, "unit": "QP-steps/s", "cores": workers, "kind": "port",
            "sample": (f"{steps} Newton steps of the oracle (reference loop order) on QPs n={n}, m={m} (3 steps "
                       f"each), {workers} single-threaded process(es) pinned one per core, ~{seconds:.0f} s each"),
            "cpu_model": model, "nproc": nproc, "cpus_available": len(avail)}


def main():
    mode = sys.argv[1]
    if mode == "step":
        out = step(*(int(a) for a in sys.argv[2:7]))
    elif mode == "batch":
        out = batch(*(int(a) if i != 2 else float(a) for i, a in enumerate(sys.argv[2:7])))
    else:
        sys.exit(f"unknown mode {mode}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
