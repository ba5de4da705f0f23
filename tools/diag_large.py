import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", d) for d in ("ipm-zoo_amd", "tests", "oracle")]
import numpy as np, torch
import ipmz_amd as I
from test_gpu_parity import _qd
print("torch stream", torch.cuda.current_stream().cuda_stream)
ctx = I.Context(0)
for N, ldpad in ((1000, 0), (1000, 24), (3000, 0), (6000, 0), (6000, 64)):
    Kh = _qd(N, 77)
    ld = N + ldpad
    Kd = torch.zeros(N, ld, dtype=torch.float64, device="cuda")
    Kd[:, :N] = torch.from_numpy(Kh).cuda()
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    info = ctx.ldlt_factor(N, Kd.data_ptr(), ld, D.data_ptr(), ws.data_ptr(), wsb)
    torch.cuda.synchronize()
    L = torch.tril(Kd[:, :N], -1) + torch.eye(N, dtype=torch.float64, device="cuda")
    rec = (L * D) @ L.T
    K = torch.from_numpy(Kh).cuda()
    ferr = (rec - K).abs().max().item()
    b = torch.rand(N, dtype=torch.float64, device="cuda") * 2 - 1
    x = b.clone()
    ctx.ldlt_solve(N, Kd.data_ptr(), ld, D.data_ptr(), ws.data_ptr(), x.data_ptr())
    torch.cuda.synchronize()
    r = (K @ x - b).abs().max().item()
    # host adapter path
    Lh, Dh, _ = I.LinearSolvers.ldlt_decomposition(Kh, ctx)
    herr = np.abs((Lh * Dh) @ Lh.T - Kh).max()
    print(f"N={N} ld={ld} info={info} factor err {ferr:.3e} solve resid {r:.3e} host-adapter factor err {herr:.3e}", flush=True)
    ctx.set_stream(None)
