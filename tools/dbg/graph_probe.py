"""Capture experiment: IPMZ_STEP_GRAPH on steps whose factor forks onto the
look-ahead streams (debug bit 4 lifts the eager fallback).  A native
backtrace is printed on SIGSEGV (tools/dbg/libsegv.so).  Prints the first
graph-replayed step's directions against an eager step from the same iterate."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import numpy as np
import torch
import ipmz_amd as I
segv = ctypes.CDLL(os.path.join(REPO, "tools", "dbg", "libsegv.so"))
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
segv.segv_install()  # after the HIP runtime's own initialisation (it may install handlers)
I.debug_inject(I.INJECT_GRAPH_FORKS | (64 if os.environ.get('PROBE_TRACE') else 0))
sizes = [(int(a), int(b), int(c)) for a, b, c in (s.split(",") for s in sys.argv[1:])] or [(1024, 256, 128)]
for use_torch_stream in (False, True):
    ctx = I.Context(0, stream=torch.cuda.current_stream().cuda_stream) if use_torch_stream else I.Context(0)
    for (n, m, p) in sizes:
        e = I.Optimizer(n, m, p, ctx)
        e.generate(1)
        g = I.Optimizer(n, m, p, ctx)
        g.generate(1)
        print("N", n + m + p, "blocking", ctx.blocking(n + m + p), "torch stream", use_torch_stream, flush=True)
        e.step(1)
        print("eager ok", flush=True)
        print("capturing", flush=True)
        g.step(3)
        print("graph captured + replayed", flush=True)
        ctx.sync()
        for which in (1, 2):
            d = np.abs(e._state(which) - g._state(which)).max()
            print("  which", which, "max |eager - graph|", d, flush=True)
        for _ in range(3):
            e.step(1)
            g.step(3)
        ctx.sync()
        print("  after 4 steps: max |eager - graph| vars", np.abs(e.vars() - g.vars()).max(), flush=True)
        e.close(); g.close()
print("graph probe done", flush=True)
