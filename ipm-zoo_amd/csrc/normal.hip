// Normal-equations reduction of the augmented KKT system (BASELINE config C2;
// the reference builds it symbolically, SymbolicOptimization.cpp:465-478,
// Optimizer.cpp:39-40, but never evaluates it -- SURVEY.md §0.4).
//
// With K = [[H, B^T], [B, -E]] (H = Q + Y^-1 L_y + Z^-1 L_z SPD, B = [A; C],
// E = diag((G^-1 L_g + H_h^-1 L_h)^-1, delta^2) > 0), K [x; l] = [r0; r1] is
//   S l = B H^{-1} r0 - r1,   S = E + B H^{-1} B^T   (SPD),
//   x   = H^{-1} (r0 - B^T l).
// The four steps of the normal equations -- Cholesky of H (as L D L^T, D > 0),
// the triangular solve L21 = B L^{-T} D^{-1}, the rank-n update S = E +
// L21 D L21^T and the Cholesky of S -- are exactly the blocked LDL^T of K with
// the x pivots first: the panel-rows kernel's TRSM with L_jj^{-1} IS the TRSM
// of B, the trailing update of the (2,2) block IS the SYRK, and the pivots
// n.. are those of -S.  capi.cpp therefore runs them as ONE pipelined factor
// (ldlt.hip / panel.hip: look-ahead, the H and S chains back to back, the
// TRSM and SYRK as MFMA strip / trailing tiles overlapping the chain) instead
// of four phases with a sequential 16-step TRSM between two factors; the
// solve is the factor's two sweeps over [r0; r1].  This file holds the
// definiteness check: H's pivots > 0 and S's (the augmented pivots n..) < 0,
// reported like a non-finite pivot: 1-based index in the augmented numbering.
#include "common.h"
#include "kernels.h"

namespace ipmz {

namespace {
constexpr int NNT = 256;
}

// info <- min(index + 1) over sign * D[i] <= 0 or non-finite
__global__ void k_ne_check_sign(const double* __restrict__ D, int N, int offset, double sign, int* __restrict__ info) {
  const int i = blockIdx.x * NNT + threadIdx.x;
  if (i < N) {
    const double v = sign * D[i];
    if (!(v > 0.0 && v <= 1.7976931348623157e308)) atomicMin(info, offset + i + 1);
  }
}

hipError_t ne_check_sign(const double* D, int N, int offset, double sign, int* info, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ne_check_sign, dim3((N + NNT - 1) / NNT), dim3(NNT), 0, st, D, N, offset, sign, info);
  return hipGetLastError();
}

}  // namespace ipmz
