"""the device-memory factor (ipmz_ldlt_factor, the
LinearSolvers entry point) on the context's own high-priority stream vs on
torch's current stream (the panel chain then runs at the caller's priority).
    python tools/factor_stream_ab.py [N ...]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("IPMZ_PKG_DIR") or os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I

torch.cuda.set_device(0)


def qd(N, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n1 = (3 * N) // 4
    K = torch.rand(N, N, device="cuda", dtype=torch.float64, generator=g) * 2 - 1
    K[:n1, :n1] /= n1
    K[n1:, :n1] /= n1 ** 0.5
    K[n1:, n1:] = 0
    idx = torch.arange(N, device="cuda")
    d = torch.rand(N, device="cuda", dtype=torch.float64, generator=g) + 0.5
    K[idx[:n1], idx[:n1]] = 1 + d[:n1]
    K[idx[n1:], idx[n1:]] = -d[n1:]
    return torch.tril(K).contiguous()


for N in [int(a) for a in sys.argv[1:]] or [2560, 11264]:
    K = qd(N, N)
    for mode in ("own", "torch", "own", "torch"):
        ctx = I.Context(0, stream=torch.cuda.current_stream().cuda_stream if mode == "torch" else None)
        wsb = ctx.workspace_bytes(N)
        ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
        D = torch.zeros(N, dtype=torch.float64, device="cuda")
        Kf = torch.empty_like(K)
        ts = []
        for it in range(8):
            Kf.copy_(K)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            assert ctx.ldlt_factor(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb) == 0  # synchronous
            ts.append(time.perf_counter() - t0)
        ts = sorted(ts[2:])
        print(f"N={N} {mode:5s}: factor {1e3 * ts[len(ts) // 2]:.3f} ms (median of 6, host-timed)", flush=True)
        ctx.close()
