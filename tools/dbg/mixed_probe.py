import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I
torch.cuda.set_device(0)
ctx = I.Context(0, stream=torch.cuda.current_stream().cuda_stream)
for N in [int(a) for a in sys.argv[1:]]:
    g = torch.Generator(device="cuda").manual_seed(N)
    K = (torch.rand(N, N, dtype=torch.float64, device="cuda", generator=g) * 2 - 1) / N
    K = torch.tril(K) + torch.tril(K, -1).T
    K.diagonal().copy_(1 + torch.rand(N, dtype=torch.float64, device="cuda", generator=g))
    wsb = ctx.mixed_workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    t = time.time()
    try:
        rc = ctx.mixed_factor(N, K.data_ptr(), N, ws.data_ptr(), wsb)
        print(N, "mixed factor rc", rc, f"{time.time()-t:.3f}s", flush=True)
    except Exception as e:
        print(N, "mixed factor FAILED", e, f"{time.time()-t:.3f}s", flush=True)
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    t = time.time()
    try:
        rc = ctx.ldlt_factor(N, K.clone().data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb)
        print(N, "f64 factor rc", rc, f"{time.time()-t:.3f}s", flush=True)
    except Exception as e:
        print(N, "f64 factor FAILED", e, f"{time.time()-t:.3f}s", flush=True)
