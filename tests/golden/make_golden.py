#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the compiled reference.

Run in the build container (where /root/reference exists):

    make -C oracle -f Makefile.ref          # builds oracle/_ref/ref_harness
    python tests/golden/make_golden.py

The harness (oracle/ref_harness.cpp) links the reference's own objects
(clang++ -O3 -DNDEBUG -ffp-contract=off) and calls
LinearSolvers::ldlt_decomposition / overwriting_solve_ldlt /
symmetric_indefinite_factorization and the Optimizer's private Newton-step
methods (Optimizer.cpp:127-219).  Outputs are raw little-endian float64
files plus manifest.json (shapes, seeds, sha256) -- data only, no reference
source is copied.
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")

CASES = [
    # (mode, args..., tag)
    ("ldlt", 8, 11, "ldlt8"),
    ("ldlt", 64, 12, "ldlt64"),
    ("ldlt", 320, 13, "ldlt320"),
    ("bk", 8, 21, "bk8"),
    ("bk", 64, 22, "bk64"),
    # dense indefinite, small diagonal: interchanges + 2x2 pivots; bkz16 has two
    # zero columns (zero-column branch + the kp = 0 defect)
    ("bk_rand", 8, 31, 0, "bkr8"),
    ("bk_rand", 64, 32, 0, "bkr64"),
    ("bk_rand", 200, 33, 0, "bkr200"),
    ("bk_rand", 16, 34, 2, "bkz16"),
    # zero column 0 plus later zero columns: the reference's 0-based info stays
    # 0 after column 0, so column 5 takes kp = 5 and column 9 the kp = 0 defect
    ("bk_zeros_at", 16, 35, "0,5,9", "bkz0_16"),
    # C1: box-only SlackedSlacks, n=64, seed 1234, full solve trace
    ("newton", 64, 0, 1234, 100, "c1"),
    # C4-size QP: n=256, m=64 (N=320), seed 0, iterates 0-3
    ("newton", 256, 64, 0, 4, "c4"),
    # small box+ineq QP, full solve
    ("newton", 48, 16, 7, 100, "s1"),
    # C3 structure, component level (Regularization equalities)
    ("component_eq", 64, 16, 8, 1234, "eq64"),
    # other Settings (newton <n> <m> <seed> <iters> <inequality handling> <inequality bounds> <variable bounds>):
    # one-sided / absent bounds -- every one converges in the reference
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Both", "Lower", "vlo"),
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Both", "Upper", "vup"),
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Both", "None", "vnone"),
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Lower", "Both", "alo"),
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Upper", "Both", "aup"),
    ("newton", 48, 0, 7, 100, "SlackedSlacks", "None", "Lower", "vlo0"),
    # InequalityHandling::Slacks: runs but stagnates (SURVEY.md App. C.1 corrector defect); 12 iterations
    ("newton", 48, 16, 7, 12, "Slacks", "Both", "Both", "sl"),
    ("newton", 48, 0, 7, 12, "Slacks", "None", "Both", "slbox"),
    # equality rows (p = 8) and the other handlings (+ <p> <equality handling>); the
    # harness expands the scalar blocks the reference's evaluate_matrix asserts on
    # (-delta^2 I, the zero lambda_A / lambda_C block), every other value is the
    # reference's own
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Both", "Both", 8, "Regularization", "reg"),
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Both", "Both", 8, "PenaltyFunction", "pen"),
    ("newton", 48, 16, 7, 100, "SlackedSlacks", "Both", "Both", 8, "SlackedSlacks", "eqss"),
    ("newton", 48, 16, 7, 100, "NaiveSlacks", "Both", "Both", 0, "none", "naive"),
    ("newton", 48, 16, 7, 100, "NaiveSlacks", "Both", "Both", 8, "Regularization", "naivereg"),
    ("newton", 48, 16, 7, 100, "NaiveSlacks", "Both", "Both", 8, "NaiveSlacks", "naiveeq"),
]


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build oracle/_ref/ref_harness first: make -C oracle -f Makefile.ref")
    subprocess.run([HARNESS, "formulation", HERE], check=True)
    for case in CASES:
        mode, tag = case[0], case[-1]
        if mode == "newton" and len(case) in (9, 11):
            # harness order: ... <iters> <tag> <ineq> <ineq bounds> <var bounds> [<p> <equality handling>]
            args = [HARNESS, mode, HERE] + [str(a) for a in case[1:5]] + [tag] + [str(a) for a in case[5:-1]]
        else:
            args = [HARNESS, mode, HERE] + [str(a) for a in case[1:-1]] + [tag]
        subprocess.run(args, check=True)
    manifest = {
        "generator": "tests/golden/make_golden.py via oracle/ref_harness.cpp",
        "reference": "albfre/ipm-zoo @ 2025-07-04 (/root/reference), clang++ -std=c++20 -O3 -DNDEBUG -ffp-contract=off",
        "clang": subprocess.run(["/opt/rocm/llvm/bin/clang++", "--version"], capture_output=True,
                                text=True).stdout.splitlines()[0],
        "cases": [list(map(str, c)) for c in CASES],
        "files": {},
    }
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".bin") or f.endswith(".txt"):
            with open(os.path.join(HERE, f), "rb") as fh:
                data = fh.read()
            manifest["files"][f] = {"bytes": len(data), "sha256": hashlib.sha256(data).hexdigest()}
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    total = sum(v["bytes"] for v in manifest["files"].values())
    print(f"wrote {len(manifest['files'])} fixture files, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
