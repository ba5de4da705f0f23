"""Run-to-run bitwise determinism of the C4 batch step (B = 1024, n = 256, m = 64).

For each factor kernel, R batches generated from the same seed take the same
eager steps; every batch's scalars and every QP's iterate and directions must
match the first batch's bitwise.  Prints the first difference found per step.
Usage: python tools/det_step.py [R] [steps] [kernels...]
"""
import sys

import numpy as np

import ipmz_amd as I

R = int(sys.argv[1]) if len(sys.argv) > 1 else 6
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
KERNELS = [int(k) for k in sys.argv[3:]] or [0, 1]  # IPMZ_BATCH_FACTOR_AUTO (left, wave-specialized at N = 320), _ONE
N_, M_, B_ = 256, 64, 1024


def snapshot(b):
    st = [b.batch_scalars().copy()]
    for w in (0, 1, 2):
        st.append(np.stack([b.state(i, w) for i in range(B_)]))
    return st


ctx = I.Context(0)
for kern in KERNELS:
    bats = []
    for r in range(R):
        b = I.Batch(N_, M_, 0, B_, ctx)
        b.set_factor_kernel(kern)
        b.generate(0)
        bats.append(b)
    bad = 0
    for it in range(STEPS):
        snaps = []
        for b in bats:
            b.step(I.STEP_RESTART_IF_CONVERGED)
            ctx.sync()
            snaps.append(snapshot(b))
        for r in range(1, R):
            for k, (x, y) in enumerate(zip(snaps[0], snaps[r])):
                if not np.array_equal(x, y):
                    rows = np.unique(np.nonzero(x != y)[0])
                    print(f"{kern} step {it} batch {r} part {k}: {len(rows)} QPs differ, first {rows[:8]}, "
                          f"max |d| {np.abs(x - y).max():.3e}", flush=True)
                    bad += 1
    print(f"{kern}: {bad} differing (step, batch, part) triples over {STEPS} steps x {R - 1} batches", flush=True)
    del bats
