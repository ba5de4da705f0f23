"""Runs tools/dbg/libcapture_probe.so (the product factor's fork/join under
hipStreamBeginCapture) on the HIP runtime torch bundles (loaded first), or on
/opt/rocm's with --no-torch.  Args: N NBO DBG."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "--no-torch" not in sys.argv:
    import torch
    torch.zeros(1, device="cuda")
    print("torch HIP", torch.version.hip, flush=True)
args = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [1408, 256, 0]
segv = ctypes.CDLL(os.path.join(REPO, "tools", "dbg", "libsegv.so"))
segv.segv_install()
lib = ctypes.CDLL(os.path.join(REPO, "tools", "dbg", "libcapture_probe.so"))
sys.exit(lib.capture_probe(*args))
