"""Readers for the committed golden fixtures (tests/golden/, see make_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.fromfile(os.path.join(GOLDEN, name), dtype="<f8")


def unpack_lower(packed, N):
    """Row-major packed lower triangle -> full symmetric (or lower) matrix."""
    M = np.zeros((N, N))
    M[np.tril_indices(N)] = packed
    return M


def sym_from_lower(packed, N):
    L = unpack_lower(packed, N)
    return L + np.tril(L, -1).T


def trace(tag):
    """Parse <tag>_trace.txt -> (variables, [iteration dicts], converged_iter|None)."""
    rows, conv = [], None
    with open(os.path.join(GOLDEN, f"{tag}_trace.txt")) as fh:
        header = fh.readline().split()[1:]
        for line in fh:
            t = line.split()
            if not t:
                continue
            if t[0] == "converged":
                conv = int(t[1])
                continue
            rows.append({t[i]: float(t[i + 1]) for i in range(2, len(t), 2)})
    return header, rows, conv
