"""Races in the factor show as run-to-run differences: the factor's
arithmetic is fixed whatever workgroup runs which role, so repeated factors of
one matrix must be bitwise identical.  Factors the same matrix R times (fp32
mixed-precision factor and fp64 factor) and reports, per repetition, the
first differing row/column of L and D against repetition 0 (-> outer panel,
inner block)."""
import os, sys
REPO = os.environ.get("PROBE_REPO") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import numpy as np
import torch
import ipmz_amd as I
torch.cuda.set_device(0)
ctx = I.Context(0)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
R = int(os.environ.get("REPS", "6"))


def qd(N, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n1 = (3 * N) // 4
    K = (torch.rand(N, N, device="cuda", dtype=torch.float64, generator=g) * 2 - 1)
    K[:n1, :n1] /= n1
    K[n1:, :n1] /= n1 ** 0.5
    K[n1:, n1:] = 0
    d = torch.rand(N, device="cuda", dtype=torch.float64, generator=g) + 0.5
    idx = torch.arange(N, device="cuda")
    K[idx[:n1], idx[:n1]] = 1 + d[:n1]
    K[idx[n1:], idx[n1:]] = -d[n1:]
    return torch.tril(K).contiguous()


def report(tag, N, nbo, Ls, Ds):
    L0, D0 = Ls[0], Ds[0]
    for r in range(1, len(Ls)):
        dl = (Ls[r] != L0) & ~(torch.isnan(Ls[r]) & torch.isnan(L0))
        dd = (Ds[r] != D0) & ~(torch.isnan(Ds[r]) & torch.isnan(D0))
        nl, nd = int(dl.sum()), int(dd.sum())
        msg = f"{tag} N={N} rep {r}: {nl} L and {nd} D elements differ"
        if nl:
            ij = torch.nonzero(dl)
            i0 = ij[:, 0].min().item()
            j0 = ij[:, 1].min().item()
            jrow = ij[ij[:, 0] == i0][:, 1].min().item()
            msg += (f"; first row {i0} (panel {i0 // nbo}, block {(i0 % nbo) // 64}) at col {jrow}; "
                    f"min col {j0} (panel {j0 // nbo}, block {(j0 % nbo) // 64}); "
                    f"nan {int(torch.isnan(Ls[r]).sum())}")
        print(msg, flush=True)


MODES = [int(m) for m in os.environ.get("MODES", "0").split(",")]
for mode, N in [(m, int(a)) for m in MODES for a in (sys.argv[1:] or [4096, 16384])]:
    I.debug_inject(mode)
    print(f"--- debug mode {mode}", flush=True)
    K = qd(N, N)
    nbo = ctx.blocking(N)[0]
    # fp32 mixed-precision factor: K32 (first in the workspace) and D32 after it
    wsb = ctx.mixed_workspace_bytes(N)
    ws = torch.zeros(wsb // 4 + 64, dtype=torch.float32, device="cuda")
    ld32 = (N + 63) // 64 * 64
    koff = 0
    doff = ((N * ld32 * 4 + 255) // 256 * 256) // 4
    Ls, Ds = [], []
    for r in range(R):
        ws.zero_()
        ctx.mixed_factor(N, K.data_ptr(), N, ws.data_ptr(), wsb)
        torch.cuda.synchronize()
        Ls.append(torch.tril(ws[koff:koff + N * ld32].view(N, ld32)[:, :N], -1).clone())
        Ds.append(ws[doff:doff + N].clone())
    report("fp32", N, nbo, Ls, Ds)
    del Ls, Ds, ws
    # fp64 factor
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    Ls, Ds = [], []
    for r in range(R):
        Kf = K.clone()
        ctx.ldlt_factor(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb)
        torch.cuda.synchronize()
        Ls.append(torch.tril(Kf, -1))
        Ds.append(D.clone())
    report("fp64", N, nbo, Ls, Ds)
    del Ls, Ds, ws, K
    torch.cuda.empty_cache()
I.debug_inject(0)
print("determinism probe done", flush=True)
