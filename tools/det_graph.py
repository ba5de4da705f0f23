"""Graph replay vs eager, C4 batch (B = 1024, n = 256, m = 64), repeated.

Each trial steps three batches from the same seed with
STEP_RESTART_IF_CONVERGED: one replaying its captured graph (as bench.py and
tests/test_gpu_c4_batch.py::test_c4_graph_replay_vs_eager_and_oracle), two
eagerly, and compares all three bitwise after every step (scalars, every QP's
iterate and both directions), printing which batch is the odd one out and
where.  Usage: python tools/det_graph.py [trials] [steps] [kernel]
"""
import sys

import numpy as np

import ipmz_amd as I

TRIALS = int(sys.argv[1]) if len(sys.argv) > 1 else 8
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 12
KERN = int(sys.argv[3]) if len(sys.argv) > 3 else 0
N_, M_, B_ = 256, 64, 1024
PARTS = ("scalars", "vars", "daff", "dir")


def snapshot(b):
    st = [b.batch_scalars().copy()]
    for w in (0, 1, 2):
        st.append(np.stack([b.state(i, w) for i in range(B_)]))
    return st


def diff(a, b):
    out = []
    for k, (x, y) in enumerate(zip(a, b)):
        if not np.array_equal(x, y):
            rows, cols = np.nonzero(x != y)
            out.append(f"{PARTS[k]}: {len(np.unique(rows))} QPs (first {np.unique(rows)[:6]}), "
                       f"cols {np.unique(cols)[:8]}, max |d| {np.abs(x - y).max():.3e}")
    return out


ctx = I.Context(0)
bad_trials = 0
for trial in range(TRIALS):
    bats = [I.Batch(N_, M_, 0, B_, ctx) for _ in range(3)]
    for b in bats:
        b.set_factor_kernel(KERN)
        b.generate(0)
    bad = False
    for it in range(STEPS):
        bats[0].step(I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH)
        bats[1].step(I.STEP_RESTART_IF_CONVERGED)
        bats[2].step(I.STEP_RESTART_IF_CONVERGED)
        ctx.sync()
        s = [snapshot(b) for b in bats]
        for (p, q) in ((0, 1), (0, 2), (1, 2)):
            d = diff(s[p], s[q])
            if d:
                bad = True
                print(f"trial {trial} step {it}: batch {p} vs {q}: " + "; ".join(d), flush=True)
        if bad:
            break
    bad_trials += bad
    print(f"trial {trial}: {'MISMATCH' if bad else 'ok'}", flush=True)
    del bats
print(f"{bad_trials} of {TRIALS} trials mismatched (kernel {KERN})", flush=True)
