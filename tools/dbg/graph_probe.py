import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I
ctypes.CDLL(os.path.join(REPO, "tools", "dbg", "libsegv.so"))
torch.cuda.set_device(0)
for use_torch_stream in (False, True):
    ctx = I.Context(0, stream=torch.cuda.current_stream().cuda_stream) if use_torch_stream else I.Context(0)
    for (n, m, p) in ((64, 16, 8), (1024, 256, 128)):
        qp = I.Optimizer(n, m, p, ctx)
        qp.generate(1)
        print("eager", use_torch_stream, n, flush=True); qp.step(1); print(qp.scalars()["alpha"], flush=True)
        print("graph", use_torch_stream, n, flush=True); qp.step(3); print(qp.scalars()["alpha"], flush=True)
        qp.step(3); torch.cuda.synchronize(); print("graph ok", flush=True)
