"""Capture repros on the HIP runtime torch bundles (loaded first):
  repro_torch.py NPAN VARIANT   tools/dbg/libgraph_fork_repro.so (the factor's pattern, trivial kernels)
  repro_torch.py mini WHICH     tools/dbg/libgraph_mini.so (minimal patterns)"""
import ctypes, os, sys
import torch
torch.zeros(1, device="cuda")
d = os.path.dirname(os.path.abspath(__file__))
if sys.argv[1] == "mini":
    sys.exit(ctypes.CDLL(os.path.join(d, "libgraph_mini.so")).mini(int(sys.argv[2])))
sys.exit(ctypes.CDLL(os.path.join(d, "libgraph_fork_repro.so")).repro(int(sys.argv[1]), int(sys.argv[2])))
