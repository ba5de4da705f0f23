"""Time the Bunch-Kaufman factor kernels (one workgroup vs whole device) on
an indefinite KKT-shaped matrix: python tools/bk_time.py N [N ...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ipm-zoo_amd"))
import ipmz_amd as I  # noqa: E402


def kkt(n, m, seed=1):
    rng = np.random.default_rng(seed)
    H = rng.uniform(-1, 1, (n, n)) / n
    H = H + H.T + np.diag(rng.uniform(0.5, 1.5, n))
    B = rng.uniform(-1, 1, (m, n))
    K = np.zeros((n + m, n + m))
    K[:n, :n] = H
    K[n:, :n] = B
    K[:n, n:] = B.T
    return K


ctx = I.Context(0)
for N in [int(a) for a in sys.argv[1:]] or [1024, 4096, 11264]:
    K = torch.from_numpy(kkt(N - N // 5, N // 5)).cuda()
    piv = torch.zeros(N, dtype=torch.int32, device="cuda")
    for algo, name in ((ctx.BK_GRID, "grid"), (ctx.BK_WORKGROUP, "workgroup")):
        if algo == ctx.BK_WORKGROUP and N > 4096:
            continue
        best = 1e9
        for rep in range(2):
            A = K.clone()
            torch.cuda.synchronize()
            t = time.perf_counter()
            ctx.bk_factor(N, A.data_ptr(), N, piv.data_ptr(), algo=algo)
            best = min(best, time.perf_counter() - t)
        # algorithmic HBM bytes of the right-looking update: read + write of the
        # trailing triangle per step, sum_k (N-k)^2/2 * 16 B = N^3/6 * 16 B
        gb = N ** 3 / 6 * 16 / 1e9
        print(f"bk {name:9s} N={N:6d}: {best * 1e3:9.2f} ms  ({gb / best:.0f} GB/s algorithmic, "
              f"{best / N * 1e6:.2f} us per pivot step)", flush=True)
    # the solve (one workgroup, LinearSolvers.cpp:209-318) on the last factor
    b = torch.ones(N, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    ctx.bk_solve(N, A.data_ptr(), N, piv.data_ptr(), b.data_ptr())
    torch.cuda.synchronize()
    ts = time.perf_counter() - t
    print(f"bk solve     N={N:6d}: {ts * 1e3:9.2f} ms", flush=True)
    if N >= 2048:  # the solve inside the EQ None Newton step: once-per-factor prep in the factor phase
        n_, p_ = N - N // 8 - N // 16, N // 16
        g = I.Optimizer(n_, N // 8, p_, ctx, equality_handling=I.EQ_NONE)
        g.generate(1)
        g.set_timing(True)
        for _ in range(2):
            g.step()
        ph = g.phase_times()
        print(f"EQ None step N={N:6d}: factor {ph['factor'] / 2:8.2f} ms, two solves {ph['solve'] / 2:7.3f} ms per step",
              flush=True)
        g.close()
