// Newton-step kernels around the factorization: synthetic QP generation,
// build_environment's initial iterate, residual (shorthand) vectors,
// KKT assembly, augmented rhs, eliminated-variable back-substitution, ratio
// tests, mu / sigma, corrector residuals and the iterate update.
//
// Formulations (tests/golden/formulations.txt is the reference's own
// symbolic output these formulas restate): InequalityHandling::SlackedSlacks
// (default) or ::Slacks, one-sided / absent inequality and variable bounds,
// EqualityHandling Regularization / None / PenaltyFunction.  The flags are
// per QP and uniform inside a launch.  The
// element-wise formulas keep the reference evaluator's operand order
// (Evaluation.cpp:102-176) and the library is built with -ffp-contract=off,
// so they round exactly like oracle/ipmz_oracle.cpp; only the reductions
// (matvecs, norms, means) and the factor/solve change summation order.
//
// Everything here is HBM-bound O(n^2) (matvecs, assembly) or O(N) work.
#include "common.h"
#include "kernels.h"
#include "sync.h"
#include "trsv_small.h"

namespace ipmz {

namespace {
constexpr int NT = 256;
constexpr int RED_BLOCKS = 512;  // partial-reduction grid
enum : uint64_t { TAG_Q = 1, TAG_C = 2, TAG_A = 3, TAG_C_EQ = 4, TAG_D = 5 };

__device__ __forceinline__ double block_sum(double v, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < NT / 64; ++w) t += sh[w];
  return t;  // valid in thread 0
}
__device__ __forceinline__ double block_min(double v, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_min(v);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double t = 1.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < NT / 64; ++w) t = fmin(t, sh[w]);
  return t;
}
// every thread gets the result (fused per-QP kernels); deterministic order
template <int NTH>
__device__ __forceinline__ double block_allsum(double v, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < NTH / 64; ++w) t += sh[w];
  __syncthreads();  // sh reusable
  return t;
}
template <int NTH>
__device__ __forceinline__ double block_allmin(double v, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_min(v);
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double t = 1.0;
  for (int w = 0; w < NTH / 64; ++w) t = fmin(t, sh[w]);
  __syncthreads();
  return t;
}
}  // namespace

// ---------------------------------------------------------------------------
// Generator, bit-identical to the oracle's generator.  Matrices are
// written row-major with leading dimension n.
__global__ void k_gen_Q(const QPDev* __restrict__ qs, uint64_t seed0) {
  const QPDev& q = qs[blockIdx.y];
  const int n = q.n;
  const int64_t ld = q.ldn;
  const uint64_t seed = seed0 + blockIdx.y;
  double* Q = const_cast<double*>(q.Q);
  const int64_t total = (int64_t)n * n;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int64_t i = t / n, j = t % n;
    double v;
    if (i == j) v = 1.0 + ipmz_u01(seed, TAG_Q, i, i);
    else if (j < i) v = (2.0 * ipmz_u01(seed, TAG_Q, i, j) - 1.0) / (double)n;
    else v = (2.0 * ipmz_u01(seed, TAG_Q, j, i) - 1.0) / (double)n;
    Q[i * ld + j] = v;
  }
}
__global__ void k_gen_rect(const QPDev* __restrict__ qs, uint64_t seed0, int which) {
  const QPDev& q = qs[blockIdx.y];
  const int n = q.n, rows = which ? q.p_usr : q.m_usr;
  const int64_t ld = q.ldn;
  const uint64_t seed = seed0 + blockIdx.y, tag = which ? TAG_C_EQ : TAG_A;
  double* M = const_cast<double*>(which ? q.C : q.A);
  const int64_t total = (int64_t)rows * n;
  const double sn = sqrt((double)n);
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int64_t i = t / n, j = t % n;
    M[i * ld + j] = (2.0 * ipmz_u01(seed, tag, i, j) - 1.0) / sn;
  }
}
__global__ void k_gen_vec(const QPDev* __restrict__ qs, uint64_t seed0) {
  const QPDev& q = qs[blockIdx.y];
  const int n = q.n, m = q.m_usr, p = q.p_usr;
  const uint64_t seed = seed0 + blockIdx.y;
  double *c = const_cast<double*>(q.c), *lA = const_cast<double*>(q.lA), *uA = const_cast<double*>(q.uA);
  double *d = const_cast<double*>(q.d), *lx = const_cast<double*>(q.lx), *ux = const_cast<double*>(q.ux);
  const int t = blockIdx.x * NT + threadIdx.x;
  if (t < n) {
    c[t] = 2.0 * ipmz_u01(seed, TAG_C, t, 0) - 1.0;
    lx[t] = -1.0;
    ux[t] = 1.0;
  }
  if (t < m) {
    lA[t] = -1.0;
    uA[t] = 1.0;
  }
  if (t < p) {
    d[t] = (2.0 * ipmz_u01(seed, TAG_D, t, 0) - 1.0) * 0.1;
    if (q.eqss) lA[m + t] = uA[m + t] = d[t];  // the equality rows as l = u = d
  }
}

static inline int max3(int a, int b, int c) { return a > b ? (a > c ? a : c) : (b > c ? b : c); }

static dim3 grid2(int64_t x, int B) { return dim3((unsigned)(x < 1 ? 1 : x), (unsigned)B); }

hipError_t qp_generate(const QPBatch& qb, uint64_t seed0, hipStream_t st) {
  const QPDev& h = qb.h;
  const int64_t gq = ((int64_t)h.n * h.n + NT - 1) / NT;
  hipLaunchKernelGGL(k_gen_Q, grid2(gq < 2048 ? gq : 2048, qb.B), dim3(NT), 0, st, qb.d, seed0);
  if (h.m_usr) {
    const int64_t g = ((int64_t)h.m_usr * h.n + NT - 1) / NT;
    hipLaunchKernelGGL(k_gen_rect, grid2(g < 1024 ? g : 1024, qb.B), dim3(NT), 0, st, qb.d, seed0, 0);
  }
  if (h.p_usr) {
    const int64_t g = ((int64_t)h.p_usr * h.n + NT - 1) / NT;
    hipLaunchKernelGGL(k_gen_rect, grid2(g < 1024 ? g : 1024, qb.B), dim3(NT), 0, st, qb.d, seed0, 1);
  }
  const int mx = max3(h.n, h.m_usr, h.p_usr);
  hipLaunchKernelGGL(k_gen_vec, grid2((mx + NT - 1) / NT, qb.B), dim3(NT), 0, st, qb.d, seed0);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// build_environment (EnvironmentBuilder.cpp:34-73): x = (l+u)/2, s = (l_A+u_A)/2,
// every other slack and dual 1.
__global__ void k_init_iterate(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  const int t = blockIdx.x * NT + threadIdx.x;
  if (t < q.n) {
    q.v[X][t] = 0.5 * (q.lx[t] + q.ux[t]);
    if (q.vlo) q.v[LY][t] = 1.0;
    if (q.vup) q.v[LZ][t] = 1.0;
    if (q.vlo && !q.slacks) q.v[Y][t] = 1.0;
    if (q.vup && !q.slacks) q.v[Z][t] = 1.0;
  }
  if (t < q.m) {
    if (!q.naive) {
      q.v[S][t] = (q.eqss && t >= q.m_usr) ? 1.0 : 0.5 * (q.lA[t] + q.uA[t]);  // t = 1 (EnvironmentBuilder.cpp)
      q.v[LA][t] = 1.0;
    }
    if (q.alo) q.v[LG][t] = 1.0;
    if (q.aup) q.v[LH][t] = 1.0;
    if (q.alo && !q.slacks) q.v[G][t] = 1.0;
    if (q.aup && !q.slacks) q.v[H][t] = 1.0;
  }
  if (t < q.p) {
    q.v[LC][t] = 1.0;
    if (!q.eqnone && !q.eqpen) q.v[P][t] = 1.0;
  }
  if (t == 0) q.scal[SC_MU_NEW] = 1.0;  // the environment's mu (EnvironmentBuilder.cpp:49)
}

hipError_t qp_init_iterate(const QPBatch& qb, hipStream_t st) {
  const int mx = max3(qb.h.n, qb.h.m, qb.h.p);
  hipLaunchKernelGGL(k_init_iterate, grid2((mx + NT - 1) / NT, qb.B), dim3(NT), 0, st, qb.d);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Dense matvecs (Evaluation.cpp:35-41 and the materialised transpose at
// :126-140).  MV selects Q x -> Qx, A x -> Ax, C x -> Cx; one wave per row,
// 16-byte loads; blockIdx.y = QP of the batch.
enum { MV_Q = 0, MV_A = 1, MV_C = 2 };
// one wave: sum_j r[j] x[j] (16-byte loads, two lane partials, DPP sum)
__device__ __forceinline__ double row_dot(const double* __restrict__ r, const double* __restrict__ x, int cols,
                                          int lane) {
  double s0 = 0.0, s1 = 0.0;
  int j = lane * 2;
  for (; j + 1 < cols; j += 128) {
    const double2 a = *reinterpret_cast<const double2*>(r + j);
    const double2 b = *reinterpret_cast<const double2*>(x + j);
    s0 += a.x * b.x;
    s1 += a.y * b.y;
  }
  if (j < cols) s0 += r[j] * x[j];
  return wave_sum(s0 + s1);
}
template <int MV>
__global__ __launch_bounds__(NT) void k_matvec_rows(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  const int rows = MV == MV_Q ? q.n : MV == MV_A ? q.m : q.p;
  const double* M = MV == MV_Q ? q.Q : MV == MV_A ? q.A : q.C;
  double* out = MV == MV_Q ? q.Qx : MV == MV_A ? q.Ax : q.Cx;
  const double* x = q.v[X];
  const int cols = q.n;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const double s = row_dot(M + (int64_t)row * q.ldn, x, cols, lane);
  if (lane == 0) out[row] = s;
}

// the vector A^T multiplies in r_x: lambda_A, or (lambda_h - lambda_g) for
// NaiveSlacks ("(A^T * (lambda_h - lambda_g))", formulations.txt)
__device__ __forceinline__ double a_dual(const QPDev& q, int i) {
  return q.naive ? q.v[LH][i] + (-q.v[LG][i]) : q.v[LA][i];
}

// A^T lambda_A -> ATl, C^T lambda_C -> CTl: column blocks of NT x row chunks
// of 128, deterministic two-pass (chunk partials, then an ordered sum).
constexpr int TCHUNK = IPMZ_TCHUNK;  // 32: C2's A^T (512 x 2048) in 128 workgroups, not 32
template <int MV>
__global__ __launch_bounds__(NT) void k_matvec_t_part(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.z];
  const int rows = MV == MV_A ? q.m : q.p, cols = q.n;
  const double* M = MV == MV_A ? q.A : q.C;
  const int j = blockIdx.x * NT + threadIdx.x;
  const int i0 = blockIdx.y * TCHUNK;
  if (j >= cols) return;
  const int i1 = i0 + TCHUNK < rows ? i0 + TCHUNK : rows;
  double s = 0.0;
#pragma unroll 8
  for (int i = i0; i < i1; ++i) s += M[(int64_t)i * q.ldn + j] * (MV == MV_A ? a_dual(q, i) : q.v[LC][i]);
  q.tpart[(int64_t)blockIdx.y * cols + j] = s;
}
template <int MV>
__global__ void k_sum_chunks(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  const int rows = MV == MV_A ? q.m : q.p, cols = q.n;
  const int nchunk = (rows + TCHUNK - 1) / TCHUNK;
  double* out = MV == MV_A ? q.ATl : q.CTl;
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= cols) return;
  double s = 0.0;
  for (int c = 0; c < nchunk; ++c) s += q.tpart[(int64_t)c * cols + j];
  out[j] = s;
}

template <int MV>
static void matvec_t(const QPBatch& qb, hipStream_t st) {
  const QPDev& h = qb.h;
  const int rows = MV == MV_A ? h.m : h.p;
  const int nchunk = (rows + TCHUNK - 1) / TCHUNK;
  hipLaunchKernelGGL((k_matvec_t_part<MV>), dim3((h.n + NT - 1) / NT, nchunk, qb.B), dim3(NT), 0, st, qb.d);
  hipLaunchKernelGGL((k_sum_chunks<MV>), grid2((h.n + NT - 1) / NT, qb.B), dim3(NT), 0, st, qb.d);
}

// number of complementarity rows (get_mu_'s divisor, Optimizer.cpp:250-268)
__device__ __forceinline__ int comp_count(const QPDev& q) { return (q.vlo + q.vup) * q.n + (q.alo + q.aup) * q.m; }

// ---------------------------------------------------------------------------
// Shorthand residuals r_v := -rhs_v at mu (SymbolicOptimization.cpp:480-492),
// plus per-block partials of ||rhs||^2, sum |complementarity|, and the two
// objective sums (Optimizer.cpp:128-130).
// one element t of the residual pass (t < n + m + p).  SC: the matvec
// results (Qx, A^T lambda_A, ...) were stored write-through by other
// workgroups of the same launch -- read them with agent-scope loads.
template <bool SC = false>
__device__ __forceinline__ void residual_elem(const QPDev& q, int t, double mu, double& res2, double& comp,
                                              double& fa, double& fb) {
  const int n = q.n, m = q.m, p = q.p;
  auto mv = [](const double* a) { return SC ? ld_sc1(a) : *a; };
  if (t < n) {
    const int i = t;
    // r_x := (c [+ lambda_z] + (Q*x) [+ (A^T*lambda_A)] [+ (C^T*lambda_C)] [- lambda_y])
    double s = q.c[i];
    if (q.vup) s = s + q.v[LZ][i];
    s = s + mv(&q.Qx[i]);
    if (m) s = s + mv(&q.ATl[i]);
    if (p) s = s + mv(&q.CTl[i]);
    const double rx = q.vlo ? s + (-q.v[LY][i]) : s;
    q.r[X][i] = rx;
    res2 += rx * rx;
    if (q.slacks) {  // (((X - L_x)*lambda_y) - (mu*e_x)), (((U_x - X)*lambda_z) - (mu*e_x))
      if (q.vlo) {
        const double r = ((q.v[X][i] + (-q.lx[i])) * q.v[LY][i]) + (-(mu * 1.0));
        q.r[LY][i] = r;
        res2 += r * r;
        comp += fabs(r);
      }
      if (q.vup) {
        const double r = ((q.ux[i] + (-q.v[X][i])) * q.v[LZ][i]) + (-(mu * 1.0));
        q.r[LZ][i] = r;
        res2 += r * r;
        comp += fabs(r);
      }
    } else {
      if (q.vlo) {
        const double rly = (q.lx[i] + q.v[Y][i]) + (-q.v[X][i]);     // (l_x + y - x)
        const double ry = q.v[Y][i] * q.v[LY][i] + (-(mu * 1.0));  // ((Y*lambda_y) - (mu*e_x))
        q.r[LY][i] = rly;
        q.r[Y][i] = ry;
        res2 += rly * rly + ry * ry;
        comp += fabs(ry);
      }
      if (q.vup) {
        const double rlz = (q.v[X][i] + q.v[Z][i]) + (-q.ux[i]);   // (x + z - u_x)
        const double rz = q.v[Z][i] * q.v[LZ][i] + (-(mu * 1.0));
        q.r[LZ][i] = rlz;
        q.r[Z][i] = rz;
        res2 += rlz * rlz + rz * rz;
        comp += fabs(rz);
      }
    }
    fa += (0.5 * q.v[X][i]) * mv(&q.Qx[i]);
    fb += q.c[i] * q.v[X][i];
  } else if (t < n + m && q.naive) {
    const int i = t - n;
    const double ax = mv(&q.Ax[i]);
    const double rlg = (q.lA[i] + q.v[G][i]) + (-ax);             // (l_A + g - (A*x))
    const double rlh = (q.v[H][i] + ax) + (-q.uA[i]);             // (h + (A*x) - u_A)
    const double rg = q.v[G][i] * q.v[LG][i] + (-(mu * 1.0));     // ((G*lambda_g) - (mu*e_A))
    const double rh = q.v[H][i] * q.v[LH][i] + (-(mu * 1.0));
    q.r[LG][i] = rlg;
    q.r[LH][i] = rlh;
    q.r[G][i] = rg;
    q.r[H][i] = rh;
    res2 += rlg * rlg + rlh * rlh + rg * rg + rh * rh;
    comp += fabs(rg) + fabs(rh);
  } else if (t < n + m) {
    const int i = t - n;
    const double rla = mv(&q.Ax[i]) + (-q.v[S][i]);  // ((A*x) - s)
    double rs;
    if (q.alo && q.aup) rs = -((q.v[LA][i] + q.v[LG][i]) + (-q.v[LH][i]));  // -(lambda_A + lambda_g - lambda_h)
    else if (q.alo) rs = -(q.v[LA][i] + q.v[LG][i]);                        // -(lambda_A + lambda_g)
    else rs = q.v[LH][i] + (-q.v[LA][i]);                                   // (lambda_h - lambda_A)
    q.r[LA][i] = rla;
    q.r[S][i] = rs;
    res2 += rla * rla + rs * rs;
    if (q.slacks) {  // (((S - L_A)*lambda_g) - (mu*e_A)), (((U_A - S)*lambda_h) - (mu*e_A))
      const double rlg = ((q.v[S][i] + (-q.lA[i])) * q.v[LG][i]) + (-(mu * 1.0));
      const double rlh = ((q.uA[i] + (-q.v[S][i])) * q.v[LH][i]) + (-(mu * 1.0));
      q.r[LG][i] = rlg;
      q.r[LH][i] = rlh;
      res2 += rlg * rlg + rlh * rlh;
      comp += fabs(rlg) + fabs(rlh);
    } else {
      if (q.alo) {
        const double rlg = (q.lA[i] + q.v[G][i]) + (-q.v[S][i]);  // (l_A + g - s)
        const double rg = q.v[G][i] * q.v[LG][i] + (-(mu * 1.0));
        q.r[LG][i] = rlg;
        q.r[G][i] = rg;
        res2 += rlg * rlg + rg * rg;
        comp += fabs(rg);
      }
      if (q.aup) {
        const double rlh = (q.v[H][i] + q.v[S][i]) + (-q.uA[i]);  // (h + s - u_A)
        const double rh = q.v[H][i] * q.v[LH][i] + (-(mu * 1.0));
        q.r[LH][i] = rlh;
        q.r[H][i] = rh;
        res2 += rlh * rlh + rh * rh;
        comp += fabs(rh);
      }
    }
  } else {
    const int i = t - n - m;
    if (q.eqnone) {  // ((C*x) - d)
      const double rlc = mv(&q.Cx[i]) + (-q.d[i]);
      q.r[LC][i] = rlc;
      res2 += rlc * rlc;
    } else if (q.eqpen) {  // -(d + (mu*lambda_C) - (C*x))
      const double rlc = -((q.d[i] + mu * q.v[LC][i]) + (-mv(&q.Cx[i])));
      q.r[LC][i] = rlc;
      res2 += rlc * rlc;
    } else {  // ((C*x) + (delta*p) - d), (p + (delta*lambda_C))
      const double rlc = (mv(&q.Cx[i]) + q.delta * q.v[P][i]) + (-q.d[i]);
      const double rp = q.v[P][i] + q.delta * q.v[LC][i];
      q.r[LC][i] = rlc;
      q.r[P][i] = rp;
      res2 += rlc * rlc + rp * rp;
    }
  }
}

__global__ __launch_bounds__(NT) void k_residuals(const QPDev* __restrict__ qs, double mu, int with_stats) {
  const QPDev& q = qs[blockIdx.y];
  __shared__ double sh[NT / 64];
  double res2 = 0.0, comp = 0.0, fa = 0.0, fb = 0.0;
  const int total = q.n + q.m + q.p;
  for (int t = blockIdx.x * NT + threadIdx.x; t < total; t += gridDim.x * NT)
    residual_elem(q, t, mu, res2, comp, fa, fb);
  if (!with_stats) return;
  double a = block_sum(res2, sh);
  if (threadIdx.x == 0) q.part[4 * blockIdx.x + 0] = a;
  a = block_sum(comp, sh);
  if (threadIdx.x == 0) q.part[4 * blockIdx.x + 1] = a;
  a = block_sum(fa, sh);
  if (threadIdx.x == 0) q.part[4 * blockIdx.x + 2] = a;
  a = block_sum(fb, sh);
  if (threadIdx.x == 0) q.part[4 * blockIdx.x + 3] = a;
}

__global__ void k_stats_final(const QPDev* __restrict__ qs, int nblocks) {
  const QPDev& q = qs[blockIdx.y];
  __shared__ double sh[4][NT];
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nblocks; b += NT)
    for (int k = 0; k < 4; ++k) s[k] += q.part[4 * b + k];
  for (int k = 0; k < 4; ++k) sh[k][threadIdx.x] = s[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < NT; ++i)
      for (int k = 0; k < 4; ++k) t[k] += sh[k][i];
    const double res = sqrt(t[0]);
    const int cnt = comp_count(q);
    const double mu = cnt == 0 ? 0.0 : t[1] / (double)cnt;
    q.scal[SC_F] = t[2] + t[3];
    q.scal[SC_RES] = res;
    q.scal[SC_MU] = mu;
    q.scal[SC_CONVERGED] = (res < 1e-8 && mu < 1e-8) ? 1.0 : 0.0;  // Optimizer.cpp:124,133
  }
}

static int red_blocks(int total) {
  int b = (total + NT - 1) / NT;
  return b < 1 ? 1 : (b > RED_BLOCKS ? RED_BLOCKS : b);
}

hipError_t qp_evaluate(const QPBatch& qb, hipStream_t st) {
  const QPDev& h = qb.h;
  hipLaunchKernelGGL((k_matvec_rows<MV_Q>), grid2((h.n + 3) / 4, qb.B), dim3(NT), 0, st, qb.d);
  if (h.m) {
    hipLaunchKernelGGL((k_matvec_rows<MV_A>), grid2((h.m + 3) / 4, qb.B), dim3(NT), 0, st, qb.d);
    matvec_t<MV_A>(qb, st);
  }
  if (h.p) {
    hipLaunchKernelGGL((k_matvec_rows<MV_C>), grid2((h.p + 3) / 4, qb.B), dim3(NT), 0, st, qb.d);
    matvec_t<MV_C>(qb, st);
  }
  const int nb = red_blocks(h.n + h.m + h.p);
  hipLaunchKernelGGL(k_residuals, grid2(nb, qb.B), dim3(NT), 0, st, qb.d, 0.0, 1);
  hipLaunchKernelGGL(k_stats_final, grid2(1, qb.B), dim3(NT), 0, st, qb.d, nb);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Augmented KKT (get_as_matrix_, Optimizer.cpp:387-391, 441-501): lower
// triangle only, row-major ld.  One workgroup per row, coalesced stores.
__device__ __forceinline__ double ds_inv(const QPDev& q, int i) {
  return ipmz_inv(ipmz_inv(q.v[G][i]) * q.v[LG][i] + ipmz_inv(q.v[H][i]) * q.v[LH][i]);
}
// Slacks: (((U_A - S)^{-1}*Lambda_h) + ((S - L_A)^{-1}*Lambda_g))^{-1}
__device__ __forceinline__ double ds_inv_sl(const QPDev& q, int i) {
  return ipmz_inv(ipmz_inv(q.uA[i] + (-q.v[S][i])) * q.v[LH][i] + ipmz_inv(q.v[S][i] + (-q.lA[i])) * q.v[LG][i]);
}
// (x, x) diagonal: Q_ii + the bound terms; (lambda_A, lambda_A) diagonal
__device__ __forceinline__ double kkt_xx(const QPDev& q, int i, double qii) {
  double h = qii;
  if (q.slacks) {  // (Q + ((U_x - X)^{-1}*Lambda_z) + ((X - L_x)^{-1}*Lambda_y))
    if (q.vup) h = h + ipmz_inv(q.ux[i] + (-q.v[X][i])) * q.v[LZ][i];
    if (q.vlo) h = h + ipmz_inv(q.v[X][i] + (-q.lx[i])) * q.v[LY][i];
  } else {  // (Q [+ (Y^{-1}*Lambda_y)] [+ (Z^{-1}*Lambda_z)])
    if (q.vlo) h = h + ipmz_inv(q.v[Y][i]) * q.v[LY][i];
    if (q.vup) h = h + ipmz_inv(q.v[Z][i]) * q.v[LZ][i];
  }
  return h;
}
__device__ __forceinline__ double kkt_aa(const QPDev& q, int i) {
  if (q.slacks) return -ds_inv_sl(q, i);
  if (q.alo && q.aup) return -ds_inv(q, i);            // -((G^{-1}*Lambda_g) + (H^{-1}*Lambda_h))^{-1}
  if (q.alo) return -(ipmz_inv(q.v[LG][i]) * q.v[G][i]);  // -(Lambda_g^{-1}*G)
  return -(ipmz_inv(q.v[LH][i]) * q.v[H][i]);             // -(Lambda_h^{-1}*H)
}

// row i of the lower triangle, columns split over nth threads (tid)
__device__ __forceinline__ void assemble_row(const QPDev& q, int i, int tid, int nth) {
  double* __restrict__ K = q.K;
  const int64_t ld = q.ldk;
  const int n = q.n, m = q.m, mk = q.mk;
  double* Kr = K + (int64_t)i * ld;
  if (i < n) {
    const double* Qr = q.Q + (int64_t)i * q.ldn;
    for (int j = tid; j < i; j += nth) Kr[j] = Qr[j];
    if (tid == 0) Kr[i] = kkt_xx(q, i, Qr[i]);
  } else if (i < n + mk && q.naive) {  // | -A | -(L_g^{-1}*G) | 0 |  and  | A | 0 | -(L_h^{-1}*H) |
    const bool hrow = i >= n + m;
    const int r = hrow ? i - n - m : i - n;
    const double* Ar = q.A + (int64_t)r * q.ldn;
    for (int j = tid; j < n; j += nth) Kr[j] = hrow ? Ar[j] : -Ar[j];
    for (int j = n + tid; j < i; j += nth) Kr[j] = 0.0;
    if (tid == 0) Kr[i] = hrow ? -(ipmz_inv(q.v[LH][r]) * q.v[H][r]) : -(ipmz_inv(q.v[LG][r]) * q.v[G][r]);
  } else if (i < n + m) {
    const int r = i - n;
    const double* Ar = q.A + (int64_t)r * q.ldn;
    for (int j = tid; j < n; j += nth) Kr[j] = Ar[j];
    for (int j = n + tid; j < i; j += nth) Kr[j] = 0.0;
    if (tid == 0) Kr[i] = kkt_aa(q, r);
  } else {
    const int r = i - n - mk;
    const double* Cr = q.C + (int64_t)r * q.ldn;
    for (int j = tid; j < n; j += nth) Kr[j] = Cr[j];
    for (int j = n + tid; j < i; j += nth) Kr[j] = 0.0;
    if (tid == 0) Kr[i] = q.eqnone ? 0.0 : q.eqpen ? -q.scal[SC_MU_NEW] : -(q.delta * q.delta);
  }
}

__global__ __launch_bounds__(NT) void k_assemble(const QPDev* __restrict__ qs) {
  assemble_row(qs[blockIdx.y], blockIdx.x, threadIdx.x, NT);
}

hipError_t qp_assemble(const QPBatch& qb, hipStream_t st) {
  hipLaunchKernelGGL(k_assemble, grid2(qb.h.N, qb.B), dim3(NT), 0, st, qb.d);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Augmented rhs (formulations.txt, augmented system rhs rows 0..2).
// element t (< N) of the augmented rhs
__device__ __forceinline__ void rhs_elem(const QPDev& q, int t) {
  const int n = q.n, m = q.m;
  if (t < n) {
    const int i = t;
    const double rx = q.r[X][i];
    if (q.slacks) {  // (((U_x - X)^{-1}*r_lz) - r_x - ((X - L_x)^{-1}*r_ly)), absent terms dropped
      double b = q.vup ? ipmz_inv(q.ux[i] + (-q.v[X][i])) * q.r[LZ][i] + (-rx) : -rx;
      if (q.vlo) b = b + (-(ipmz_inv(q.v[X][i] + (-q.lx[i])) * q.r[LY][i]));
      q.b[i] = b;
      return;
    }
    const double tz = q.vup ? ipmz_inv(q.v[Z][i]) * (q.r[Z][i] + (-(q.v[LZ][i] * q.r[LZ][i]))) : 0.0;
    const double ty = q.vlo ? ipmz_inv(q.v[Y][i]) * (q.r[Y][i] + (-(q.v[LY][i] * q.r[LY][i]))) : 0.0;
    if (q.vlo && q.vup) q.b[i] = (tz + (-rx)) + (-ty);
    else if (q.vup) q.b[i] = tz + (-rx);  // ((Z^{-1}*(r_z - (L_z*r_lz))) - r_x)
    else if (q.vlo) q.b[i] = -(rx + ty);  // -(r_x + (Y^{-1}*(r_y - (L_y*r_ly))))
    else q.b[i] = -rx;
  } else if (t < n + q.mk && q.naive) {
    if (t < n + m) {  // ((L_g^{-1}*r_g) - r_lg)
      const int i = t - n;
      q.b[t] = ipmz_inv(q.v[LG][i]) * q.r[G][i] + (-q.r[LG][i]);
    } else {  // ((L_h^{-1}*r_h) - r_lh)
      const int i = t - n - m;
      q.b[t] = ipmz_inv(q.v[LH][i]) * q.r[H][i] + (-q.r[LH][i]);
    }
  } else if (t < n + m) {
    const int i = t - n;
    const double rla = q.r[LA][i], rs = q.r[S][i];
    if (q.slacks) {
      const double a = ipmz_inv(q.uA[i] + (-q.v[S][i])) * q.r[LH][i];
      const double c = ipmz_inv(q.v[S][i] + (-q.lA[i])) * q.r[LG][i];
      q.b[t] = ds_inv_sl(q, i) * ((a + (-rs)) + (-c)) + (-rla);
    } else if (q.alo && q.aup) {
      const double th = ipmz_inv(q.v[H][i]) * (q.r[H][i] + (-(q.v[LH][i] * q.r[LH][i])));
      const double tg = ipmz_inv(q.v[G][i]) * (q.r[G][i] + (-(q.v[LG][i] * q.r[LG][i])));
      q.b[t] = ds_inv(q, i) * ((th + (-rs)) + (-tg)) + (-rla);
    } else if (q.alo) {  // -(r_lA + (L_g^{-1}*(r_g + (G*r_s))) - r_lg)
      q.b[t] = -((rla + ipmz_inv(q.v[LG][i]) * (q.r[G][i] + q.v[G][i] * rs)) + (-q.r[LG][i]));
    } else {  // ((L_h^{-1}*(r_h - (H*r_s))) - r_lA - r_lh)
      q.b[t] = ((ipmz_inv(q.v[LH][i]) * (q.r[H][i] + (-(q.v[H][i] * rs)))) + (-rla)) + (-q.r[LH][i]);
    }
  } else if (t < q.N) {
    const int i = t - n - q.mk;
    q.b[t] = (q.eqnone || q.eqpen) ? -q.r[LC][i] : q.delta * q.r[P][i] + (-q.r[LC][i]);
  }
}

__global__ void k_rhs(const QPDev* __restrict__ qs) { rhs_elem(qs[blockIdx.y], blockIdx.x * NT + threadIdx.x); }

hipError_t qp_rhs(const QPBatch& qb, hipStream_t st) {
  hipLaunchKernelGGL(k_rhs, grid2((qb.h.N + NT - 1) / NT, qb.B), dim3(NT), 0, st, qb.d);
  return hipGetLastError();
}

// Back-substitution of the eliminated variables (delta_definitions,
// Optimizer.cpp:373-378) into the affine (which = 0) or corrector (1) slots.
struct DSel {
  double* const* d;
};
__device__ __forceinline__ DSel dsel(const QPDev& q, int which) { return DSel{which ? q.dir : q.daff}; }

// element t (< N): the solution b -> the Newton directions D
__device__ __forceinline__ void backsub_elem(const QPDev& q, const DSel& D, int t) {
  const int n = q.n, m = q.m;
  if (t < n) {
    const int i = t;
    const double dx = q.b[i];
    D.d[X][i] = dx;
    if (q.slacks) {
      if (q.vlo)  // -((X - L_x)^{-1}*(r_ly + (L_y*dx)))
        D.d[LY][i] = -(ipmz_inv(q.v[X][i] + (-q.lx[i])) * (q.r[LY][i] + q.v[LY][i] * dx));
      if (q.vup)  // ((U_x - X)^{-1}*((L_z*dx) - r_lz))
        D.d[LZ][i] = ipmz_inv(q.ux[i] + (-q.v[X][i])) * (q.v[LZ][i] * dx + (-q.r[LZ][i]));
      return;
    }
    if (q.vlo) {
      D.d[LY][i] = -((ipmz_inv(q.v[Y][i]) * q.v[LY][i]) *
                     ((dx + ipmz_inv(q.v[LY][i]) * q.r[Y][i]) + (-q.r[LY][i])));
      D.d[Y][i] = -(ipmz_inv(q.v[LY][i]) * (q.r[Y][i] + q.v[Y][i] * D.d[LY][i]));
    }
    if (q.vup) {
      D.d[LZ][i] = -((ipmz_inv(q.v[Z][i]) * q.v[LZ][i]) *
                     ((ipmz_inv(q.v[LZ][i]) * q.r[Z][i] + (-q.r[LZ][i])) + (-dx)));
      D.d[Z][i] = -(ipmz_inv(q.v[LZ][i]) * (q.r[Z][i] + q.v[Z][i] * D.d[LZ][i]));
    }
  } else if (t < n + q.mk && q.naive) {
    if (t < n + m) {  // -(L_g^{-1}*(r_g + (G*dl_g)))
      const int i = t - n;
      const double dlg = q.b[t];
      D.d[LG][i] = dlg;
      D.d[G][i] = -(ipmz_inv(q.v[LG][i]) * (q.r[G][i] + q.v[G][i] * dlg));
    } else {
      const int i = t - n - m;
      const double dlh = q.b[t];
      D.d[LH][i] = dlh;
      D.d[H][i] = -(ipmz_inv(q.v[LH][i]) * (q.r[H][i] + q.v[H][i] * dlh));
    }
  } else if (t < n + m) {
    const int i = t - n;
    const double dla = q.b[t], rs = q.r[S][i];
    D.d[LA][i] = dla;
    if (q.slacks) {
      const double a = ipmz_inv(q.uA[i] + (-q.v[S][i])) * q.r[LH][i];
      const double c = ipmz_inv(q.v[S][i] + (-q.lA[i])) * q.r[LG][i];
      const double ds = ds_inv_sl(q, i) * (((dla + a) + (-rs)) + (-c));
      D.d[S][i] = ds;
      D.d[LG][i] = -(ipmz_inv(q.v[S][i] + (-q.lA[i])) * (q.r[LG][i] + q.v[LG][i] * ds));
      D.d[LH][i] = ipmz_inv(q.uA[i] + (-q.v[S][i])) * (q.v[LH][i] * ds + (-q.r[LH][i]));
      return;
    }
    double ds;
    if (q.alo && q.aup) {
      const double th = ipmz_inv(q.v[H][i]) * (q.r[H][i] + (-(q.v[LH][i] * q.r[LH][i])));
      const double tg = ipmz_inv(q.v[G][i]) * (q.r[G][i] + (-(q.v[LG][i] * q.r[LG][i])));
      ds = ds_inv(q, i) * (((dla + th) + (-rs)) + (-tg));
    } else if (q.alo) {  // (L_g^{-1}*G*(dla - r_s - (G^{-1}*(r_g - (L_g*r_lg)))))
      ds = (ipmz_inv(q.v[LG][i]) * q.v[G][i]) *
           ((dla + (-rs)) + (-(ipmz_inv(q.v[G][i]) * (q.r[G][i] + (-(q.v[LG][i] * q.r[LG][i]))))));
    } else {  // (L_h^{-1}*H*(dla + (H^{-1}*(r_h - (L_h*r_lh))) - r_s))
      ds = (ipmz_inv(q.v[LH][i]) * q.v[H][i]) *
           ((dla + ipmz_inv(q.v[H][i]) * (q.r[H][i] + (-(q.v[LH][i] * q.r[LH][i])))) + (-rs));
    }
    D.d[S][i] = ds;
    if (q.alo) {
      const double dlg =
          -((ipmz_inv(q.v[G][i]) * q.v[LG][i]) * ((ds + ipmz_inv(q.v[LG][i]) * q.r[G][i]) + (-q.r[LG][i])));
      D.d[LG][i] = dlg;
      D.d[G][i] = -(ipmz_inv(q.v[LG][i]) * (q.r[G][i] + q.v[G][i] * dlg));
    }
    if (q.aup) {
      const double dlh =
          -((ipmz_inv(q.v[H][i]) * q.v[LH][i]) * ((ipmz_inv(q.v[LH][i]) * q.r[H][i] + (-q.r[LH][i])) + (-ds)));
      D.d[LH][i] = dlh;
      D.d[H][i] = -(ipmz_inv(q.v[LH][i]) * (q.r[H][i] + q.v[H][i] * dlh));
    }
  } else if (t < q.N) {
    const int i = t - n - q.mk;
    const double dlc = q.b[t];
    D.d[LC][i] = dlc;
    if (!q.eqnone && !q.eqpen) D.d[P][i] = -(q.r[P][i] + q.delta * dlc);
  }
}

__global__ void k_backsub(const QPDev* __restrict__ qs, int which) {
  const QPDev& q = qs[blockIdx.y];
  backsub_elem(q, dsel(q, which), blockIdx.x * NT + threadIdx.x);
}

hipError_t qp_backsub(const QPBatch& qb, int which, hipStream_t st) {
  hipLaunchKernelGGL(k_backsub, grid2((qb.h.N + NT - 1) / NT, qb.B), dim3(NT), 0, st, qb.d, which);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// get_max_step_ (Optimizer.cpp:270-342): fraction-to-boundary over the
// non-negative Newton variables, plus -- when neither g nor h is a Newton
// variable (box-only SlackedSlacks, or Slacks) -- explicit bounds on x
// (l_x, u_x) and s (l_A, u_A), both always (the environment holds both).
// Element t (< n + m), folded into a.
__device__ __forceinline__ void ratio_elem(const QPDev& q, const DSel& D, int t, double& a) {
  const int n = q.n, m = q.m;
  const bool explicit_bounds = q.slacks || m == 0;
  auto nonneg = [&](int slot, int i) {
    const double d = D.d[slot][i];
    if (d < 0.0) a = fmin(a, -q.v[slot][i] / d);
  };
  auto bounded = [&](double v, double d, double lo, double up) {
    if (d < 0.0) a = fmin(a, (lo - v) / d);
    if (d > 0.0) a = fmin(a, (up - v) / d);
  };
  if (t < n) {
    const int i = t;
    if (q.vlo) nonneg(LY, i);
    if (q.vup) nonneg(LZ, i);
    if (!q.slacks) {
      if (q.vlo) nonneg(Y, i);
      if (q.vup) nonneg(Z, i);
    }
    if (explicit_bounds) bounded(q.v[X][i], D.d[X][i], q.lx[i], q.ux[i]);
  } else {
    const int i = t - n;
    if (q.alo) nonneg(LG, i);
    if (q.aup) nonneg(LH, i);
    if (!q.slacks) {
      if (q.alo) nonneg(G, i);
      if (q.aup) nonneg(H, i);
    }
    if (explicit_bounds) bounded(q.v[S][i], D.d[S][i], q.lA[i], q.uA[i]);
  }
}

__global__ __launch_bounds__(NT) void k_ratio_part(const QPDev* __restrict__ qs, int which) {
  const QPDev& q = qs[blockIdx.y];
  const DSel D = dsel(q, which);
  __shared__ double sh[NT / 64];
  double a = 1.0;
  for (int t = blockIdx.x * NT + threadIdx.x; t < q.n + q.m; t += gridDim.x * NT) ratio_elem(q, D, t, a);
  a = block_min(a, sh);
  if (threadIdx.x == 0) q.part[blockIdx.x] = a;
}
__global__ void k_min_final(const QPDev* __restrict__ qs, int nblocks, int out_index) {
  const QPDev& q = qs[blockIdx.y];
  __shared__ double sh[NT / 64];
  double a = 1.0;
  for (int b = threadIdx.x; b < nblocks; b += NT) a = fmin(a, q.part[b]);
  a = block_min(a, sh);
  if (threadIdx.x == 0) q.scal[out_index] = a;
}

hipError_t qp_ratio(const QPBatch& qb, int which, int out_index, hipStream_t st) {
  const int nb = red_blocks(qb.h.n + qb.h.m);
  hipLaunchKernelGGL(k_ratio_part, grid2(nb, qb.B), dim3(NT), 0, st, qb.d, which);
  hipLaunchKernelGGL(k_min_final, grid2(1, qb.B), dim3(NT), 0, st, qb.d, nb, out_index);
  return hipGetLastError();
}

// mu at the affine trial point v + alpha_aff * daff (Optimizer.cpp:167-180):
// |complementarity| of every row that carries e and mu, at the trial point.
__device__ __forceinline__ void mu_aff_elem(const QPDev& q, int t, double al, double& s) {
  const int n = q.n;
  auto tv = [&](int slot, int i) { return q.v[slot][i] + al * q.daff[slot][i]; };
  auto term = [&](double a, double b) { return fabs(-(a * b + (-(0.0 * 1.0)))); };
  if (t < n) {
    const int i = t;
    if (q.slacks) {
      if (q.vlo) s += term(tv(X, i) + (-q.lx[i]), tv(LY, i));  // ((X - L_x)*lambda_y)
      if (q.vup) s += term(q.ux[i] + (-tv(X, i)), tv(LZ, i));  // ((U_x - X)*lambda_z)
    } else {
      if (q.vlo) s += term(tv(Y, i), tv(LY, i));
      if (q.vup) s += term(tv(Z, i), tv(LZ, i));
    }
  } else {
    const int i = t - n;
    if (q.slacks) {
      s += term(tv(S, i) + (-q.lA[i]), tv(LG, i));  // ((S - L_A)*lambda_g)
      s += term(q.uA[i] + (-tv(S, i)), tv(LH, i));  // ((U_A - S)*lambda_h)
    } else {
      if (q.alo) s += term(tv(G, i), tv(LG, i));
      if (q.aup) s += term(tv(H, i), tv(LH, i));
    }
  }
}
__global__ __launch_bounds__(NT) void k_mu_aff_part(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  __shared__ double sh[NT / 64];
  const double al = q.scal[SC_ALPHA_AFF];
  double s = 0.0;
  for (int t = blockIdx.x * NT + threadIdx.x; t < q.n + q.m; t += gridDim.x * NT) mu_aff_elem(q, t, al, s);
  s = block_sum(s, sh);
  if (threadIdx.x == 0) q.part[blockIdx.x] = s;
}
// mu_aff, sigma = (mu_aff / mu)^3, mu_new = mu sigma (Optimizer.cpp:167-182)
__device__ __forceinline__ double mu_aff_store(const QPDev& q, double s) {
  const int cnt = comp_count(q);
  const double mu_aff = cnt == 0 ? 0.0 : s / (double)cnt;
  const double mu = q.scal[SC_MU];
  const double sigma = mu > 0.0 ? pow(mu_aff / mu, 3.0) : 0.0;
  q.scal[SC_MU_AFF] = mu_aff;
  q.scal[SC_SIGMA] = sigma;
  q.scal[SC_MU_NEW] = mu * sigma;
  return mu * sigma;
}
__global__ void k_mu_aff_final(const QPDev* __restrict__ qs, int nblocks) {
  const QPDev& q = qs[blockIdx.y];
  __shared__ double sh[NT / 64];
  double s = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += NT) s += q.part[b];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) mu_aff_store(q, s);
}

hipError_t qp_mu_aff(const QPBatch& qb, hipStream_t st) {
  const int nb = red_blocks(qb.h.n + qb.h.m);
  hipLaunchKernelGGL(k_mu_aff_part, grid2(nb, qb.B), dim3(NT), 0, st, qb.d);
  hipLaunchKernelGGL(k_mu_aff_final, grid2(1, qb.B), dim3(NT), 0, st, qb.d, nb);
  return hipGetLastError();
}

// Corrector (Optimizer.cpp:183-209): every complementarity row at mu_new plus
// the same row with mu -> 0 and every VARIABLE replaced by its affine
// direction: SlackedSlacks r_y = (Y lambda_y - mu_new e) + (dY_aff
// dlambda_y_aff - 0 e); Slacks r_lambda_y = ((X - L_x) lambda_y - mu_new e) +
// ((dX_aff - L_x) dlambda_y_aff - 0 e) -- the bound constant leaks into the
// correction (the reference's Slacks defect, SURVEY.md App. C.1, reproduced).
__device__ __forceinline__ void corrector_elem(const QPDev& q, int t, double mu) {
  const int n = q.n, m = q.m;
  const double* const* v = q.v;
  const double* const* da = q.daff;
  auto ss = [&](int c, int d, int i) {  // SlackedSlacks pair (c = slack, d = its dual)
    q.r[c][i] = (v[c][i] * v[d][i] + (-(mu * 1.0))) + (da[c][i] * da[d][i] + (-(0.0 * 1.0)));
  };
  if (t < n) {
    const int i = t;
    if (q.slacks) {
      if (q.vlo)
        q.r[LY][i] = (((v[X][i] + (-q.lx[i])) * v[LY][i]) + (-(mu * 1.0))) +
                     ((da[X][i] + (-q.lx[i])) * da[LY][i] + (-(0.0 * 1.0)));
      if (q.vup)
        q.r[LZ][i] = (((q.ux[i] + (-v[X][i])) * v[LZ][i]) + (-(mu * 1.0))) +
                     ((q.ux[i] + (-da[X][i])) * da[LZ][i] + (-(0.0 * 1.0)));
    } else {
      if (q.vlo) ss(Y, LY, i);
      if (q.vup) ss(Z, LZ, i);
    }
  } else if (t < n + m) {
    const int i = t - n;
    if (q.slacks) {
      q.r[LG][i] = (((v[S][i] + (-q.lA[i])) * v[LG][i]) + (-(mu * 1.0))) +
                   ((da[S][i] + (-q.lA[i])) * da[LG][i] + (-(0.0 * 1.0)));
      q.r[LH][i] = (((q.uA[i] + (-v[S][i])) * v[LH][i]) + (-(mu * 1.0))) +
                   ((q.uA[i] + (-da[S][i])) * da[LH][i] + (-(0.0 * 1.0)));
    } else {
      if (q.alo) ss(G, LG, i);
      if (q.aup) ss(H, LH, i);
    }
  } else {
    // PenaltyFunction: r_lambda_C carries mu (no e, so no affine correction)
    const int i = t - n - m;
    if (q.eqpen && i < q.p) q.r[LC][i] = -((q.d[i] + mu * v[LC][i]) + (-q.Cx[i]));
  }
}
__global__ void k_corrector(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  corrector_elem(q, blockIdx.x * NT + threadIdx.x, q.scal[SC_MU_NEW]);
}

hipError_t qp_corrector_residuals(const QPBatch& qb, hipStream_t st) {
  const int rows = qb.h.n + qb.h.m + (qb.h.eqpen ? qb.h.p : 0);
  hipLaunchKernelGGL(k_corrector, grid2((rows + NT - 1) / NT, qb.B), dim3(NT), 0, st, qb.d);
  return hipGetLastError();
}

// update_variables_(0.995 * alpha, ...) (Optimizer.cpp:216-231)
// freeze != 0: a converged QP of a batch keeps its iterate (the reference
// stops iterating it, Optimizer.cpp:133-135).
__device__ __forceinline__ void update_elem(const QPDev& q, int t, double s) {
  const int n = q.n, m = q.m, p = q.p;
  auto up = [&](int slot, int i) { q.v[slot][i] = q.v[slot][i] + s * q.dir[slot][i]; };
  if (t < n) {
    up(X, t);
    if (q.vlo) up(LY, t);
    if (q.vup) up(LZ, t);
    if (q.vlo && !q.slacks) up(Y, t);
    if (q.vup && !q.slacks) up(Z, t);
  }
  if (t < m) {
    if (!q.naive) {
      up(LA, t);
      up(S, t);
    }
    if (q.alo) up(LG, t);
    if (q.aup) up(LH, t);
    if (q.alo && !q.slacks) up(G, t);
    if (q.aup && !q.slacks) up(H, t);
  }
  if (t < p) {
    up(LC, t);
    if (!q.eqnone && !q.eqpen) up(P, t);
  }
}
__global__ void k_update(const QPDev* __restrict__ qs, int freeze) {
  const QPDev& q = qs[blockIdx.y];
  if (freeze && q.scal[SC_CONVERGED] != 0.0) return;
  update_elem(q, blockIdx.x * NT + threadIdx.x, 0.995 * q.scal[SC_ALPHA]);
}

hipError_t qp_update(const QPBatch& qb, int freeze, hipStream_t st) {
  const int mx = max3(qb.h.n, qb.h.m, qb.h.p);
  hipLaunchKernelGGL(k_update, grid2((mx + NT - 1) / NT, qb.B), dim3(NT), 0, st, qb.d, freeze);
  return hipGetLastError();
}

// Benchmark restart: a converged iterate is reset (on device, no host sync)
// to the saved initial state, so every timed step is a real Newton step.
__global__ void k_restart_copy(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  if (q.scal[SC_CONVERGED] == 0.0) return;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < q.state_len; t += (int64_t)gridDim.x * NT) {
    q.v[0][t] = q.v0[t];
    q.r[0][t] = q.r0[t];
  }
}
__global__ void k_restart_scal(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  if (threadIdx.x != 0 || q.scal[SC_CONVERGED] == 0.0) return;
  const double restarts = q.scal[SC_RESTARTS];
  for (int k = 0; k < SC_RESTARTS; ++k) q.scal[k] = q.scal0[k];
  q.scal[SC_RESTARTS] = restarts + 1.0;
}

hipError_t qp_restart_if_converged(const QPBatch& qb, hipStream_t st) {
  const int64_t g = (qb.h.state_len + NT - 1) / NT;
  hipLaunchKernelGGL(k_restart_copy, grid2(g < 256 ? g : 256, qb.B), dim3(NT), 0, st, qb.d);
  hipLaunchKernelGGL(k_restart_scal, grid2(1, qb.B), dim3(64), 0, st, qb.d);
  return hipGetLastError();
}

// Convergence summary of a batch (the input of the cross-GPU all-reduce,
// SURVEY.md §8e; the stopping rule res < 1e-8 and mu < 1e-8 of
// Optimizer.cpp:124-135): out = {max res, max mu, unconverged count} -- all
// three MAX-reducible, so ONE all-reduce (MAX) over the ranks decides the
// stop: every QP of the job converged <=> the reduced out[2] == 0.
__global__ __launch_bounds__(NT) void k_batch_summary(const QPDev* __restrict__ qs, int B, double* __restrict__ out) {
  __shared__ double sh[3][NT];
  double r = 0.0, m = 0.0, u = 0.0;
  for (int b = threadIdx.x; b < B; b += NT) {
    const double* sc = qs[b].scal;
    r = fmax(r, sc[SC_RES]);
    m = fmax(m, sc[SC_MU]);
    u += sc[SC_CONVERGED] != 0.0 ? 0.0 : 1.0;
  }
  sh[0][threadIdx.x] = r;
  sh[1][threadIdx.x] = m;
  sh[2][threadIdx.x] = u;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      sh[0][threadIdx.x] = fmax(sh[0][threadIdx.x], sh[0][threadIdx.x + s]);
      sh[1][threadIdx.x] = fmax(sh[1][threadIdx.x], sh[1][threadIdx.x + s]);
      sh[2][threadIdx.x] += sh[2][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x < 3) out[threadIdx.x] = sh[threadIdx.x][0];
}
hipError_t qp_batch_summary(const QPBatch& qb, double* out, hipStream_t st) {
  hipLaunchKernelGGL(k_batch_summary, dim3(1), dim3(NT), 0, st, qb.d, qb.B, out);
  return hipGetLastError();
}

// snapshot of the initial iterate (restart source)
__global__ void k_save_initial(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < q.state_len; t += (int64_t)gridDim.x * NT) {
    q.v0[t] = q.v[0][t];
    q.r0[t] = q.r[0][t];
  }
  if (blockIdx.x == 0 && threadIdx.x < SC_COUNT) q.scal0[threadIdx.x] = q.scal[threadIdx.x];
}
hipError_t qp_save_initial(const QPBatch& qb, hipStream_t st) {
  const int64_t g = (qb.h.state_len + NT - 1) / NT;
  hipLaunchKernelGGL(k_save_initial, grid2(g < 256 ? g : 256, qb.B), dim3(NT), 0, st, qb.d);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused per-QP step phases for batches of small systems (config C4): ONE
// workgroup per QP runs every O(N) / O(n^2) phase between the factor and the
// solves, so a Newton step is six launches (pre, factor, solve, mid, solve,
// post) instead of ~25 -- at 128 QPs per GPU the short grid kernels above
// were ~5 us each, a quarter of the step.  The element formulas are the
// same device functions as the grid kernels (bitwise the same values); only
// the reductions (res, comp, f, mu_aff) sum in a different order.
constexpr int FT = 512;  // 8 waves

// restart-if-converged, KKT assembly, affine rhs.  gridDim.x workgroups per
// QP (blockIdx.y): the off-diagonal copy (independent of the iterate) is
// split over all of them; workgroup 0 also restarts, writes the diagonal and
// the rhs (which read the iterate) in that order.
// kmode (kernels.h KMODE_*): where the matrix goes -- K whole, or the kept
// K0 (its off-diagonal part once per data load, its diagonal every step)
__global__ __launch_bounds__(FT) void k_fused_pre(const QPDev* __restrict__ qs, int restart, int* info, int kmode) {
  const QPDev& q = qs[blockIdx.y];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool lead = blockIdx.x == 0 && kmode != KMODE_K0_OFFDIAG;
  double* const KT = kmode == KMODE_K ? q.K : q.K0;
  if (info && lead && blockIdx.y == 0 && tid == 0) *info = 0x7f7f7f7f;  // the factor's first-failure word
  if (lead && restart && q.scal[SC_CONVERGED] != 0.0) {
    for (int64_t t = tid; t < q.state_len; t += FT) {
      q.v[0][t] = q.v0[t];
      q.r[0][t] = q.r0[t];
    }
    __syncthreads();  // every thread has read SC_CONVERGED
    if (tid == 0) {
      const double restarts = q.scal[SC_RESTARTS];
      for (int k = 0; k < SC_RESTARTS; ++k) q.scal[k] = q.scal0[k];
      q.scal[SC_RESTARTS] = restarts + 1.0;
    }
    __syncthreads();  // v, r and mu_new restored before assembly reads them
  }
  // strict lower triangle in 128-column units (a wave per unit, a column
  // pair per lane), eight units per wave in flight: one workgroup moves the
  // QP's ~0.8 MB only with many loads outstanding
  const int N = q.N, n = q.n, m = q.m, nm = q.n + q.mk;
  const int nch = (N + 127) / 128, units = kmode == KMODE_K0_DIAG ? 0 : N * nch;
  for (int u0 = (blockIdx.x * (FT / 64) + wave) * 8; u0 < units; u0 += gridDim.x * (FT / 64) * 8) {
    double v0[8], v1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int u = u0 + k, i = u / nch, j = (u % nch) * 128 + 2 * lane;
      v0[k] = v1[k] = 0.0;
      if (u < units) {
        // NaiveSlacks: the lambda_g rows hold -A, the lambda_h rows A
        const bool ah = q.naive && i >= n + m && i < nm;
        const double* src = i < n ? q.Q + (int64_t)i * q.ldn
                           : i < nm ? q.A + (int64_t)(ah ? i - n - m : i - n) * q.ldn : q.C + (int64_t)(i - nm) * q.ldn;
        const bool neg = q.naive && i >= n && i < n + m;
        const int lim = i < n ? i : n;  // source columns [0, lim); zeros in [n, i)
        if (j + 1 < lim) {  // one 16-byte load (ldn and j even)
          const double2 t = *reinterpret_cast<const double2*>(src + j);
          v0[k] = neg ? -t.x : t.x;
          v1[k] = neg ? -t.y : t.y;
        } else if (j < lim) {
          v0[k] = neg ? -src[j] : src[j];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int u = u0 + k, i = u / nch, j = (u % nch) * 128 + 2 * lane;
      if (u < units) {
        double* Kr = KT + (int64_t)i * q.ldk;
        if (j + 1 < i) *reinterpret_cast<double2*>(Kr + j) = make_double2(v0[k], v1[k]);  // ldk even
        else if (j < i) Kr[j] = v0[k];
      }
    }
  }
  if (!lead) return;
  for (int i = tid; i < N; i += FT) {
    double* Kd = KT + (int64_t)i * q.ldk + i;
    if (i < n) *Kd = kkt_xx(q, i, q.Q[(int64_t)i * q.ldn + i]);
    else if (q.naive && i < n + m) *Kd = -(ipmz_inv(q.v[LG][i - n]) * q.v[G][i - n]);
    else if (q.naive && i < nm) *Kd = -(ipmz_inv(q.v[LH][i - n - m]) * q.v[H][i - n - m]);
    else if (i < nm) *Kd = kkt_aa(q, i - n);
    else *Kd = q.eqnone ? 0.0 : q.eqpen ? -q.scal[SC_MU_NEW] : -(q.delta * q.delta);
  }
  for (int t = tid; t < N; t += FT) rhs_elem(q, t);
}

// predictor back-substitution, alpha_aff, mu_aff / sigma, corrector rows,
// corrector rhs
// (T threads per QP; sh: T / 64 doubles of LDS)
template <int T>
__device__ __forceinline__ void fused_mid_body(const QPDev& q, double* sh) {
  const int tid = threadIdx.x;
  const int N = q.N, nm = q.n + q.m;
  const DSel D = dsel(q, 0);
  for (int t = tid; t < N; t += T) backsub_elem(q, D, t);
  __syncthreads();
  double a = 1.0;
  for (int t = tid; t < nm; t += T) ratio_elem(q, D, t, a);
  a = block_allmin<T>(a, sh);
  if (tid == 0) q.scal[SC_ALPHA_AFF] = a;
  double s = 0.0;
  for (int t = tid; t < nm; t += T) mu_aff_elem(q, t, a, s);
  s = block_allsum<T>(s, sh);
  // every thread evaluates the same scalars; thread 0 stores them
  const int cnt = comp_count(q);
  const double mu_aff = cnt == 0 ? 0.0 : s / (double)cnt;
  const double mu = q.scal[SC_MU];
  const double sigma = mu > 0.0 ? pow(mu_aff / mu, 3.0) : 0.0;
  const double mu_new = mu * sigma;
  const int rows = nm + (q.eqpen ? q.p : 0);
  for (int t = tid; t < rows; t += T) corrector_elem(q, t, mu_new);
  __syncthreads();  // SC_MU read by every thread; corrector rows written
  if (tid == 0) {
    q.scal[SC_MU_AFF] = mu_aff;
    q.scal[SC_SIGMA] = sigma;
    q.scal[SC_MU_NEW] = mu_new;
  }
  for (int t = tid; t < N; t += T) rhs_elem(q, t);
}
__global__ __launch_bounds__(FT) void k_fused_mid(const QPDev* __restrict__ qs) {
  __shared__ double sh[FT / 64];
  fused_mid_body<FT>(qs[blockIdx.x], sh);
}

// corrector back-substitution, alpha, the update (one workgroup per QP)
template <int T>
__device__ __forceinline__ void fused_post_body(const QPDev& q, int freeze, double* sh) {
  const int tid = threadIdx.x;
  const int n = q.n, m = q.m, p = q.p, N = q.N;
  const DSel D = dsel(q, 1);
  const bool frozen = freeze && q.scal[SC_CONVERGED] != 0.0;
  for (int t = tid; t < N; t += T) backsub_elem(q, D, t);
  __syncthreads();
  double a = 1.0;
  for (int t = tid; t < n + m; t += T) ratio_elem(q, D, t, a);
  a = block_allmin<T>(a, sh);
  if (tid == 0) q.scal[SC_ALPHA] = a;
  if (!frozen) {
    const int mx = max(n, max(m, p));
    for (int t = tid; t < mx; t += T) update_elem(q, t, 0.995 * a);
  }
}
__global__ __launch_bounds__(FT) void k_fused_post(const QPDev* __restrict__ qs, int freeze) {
  __shared__ double sh[FT / 64];
  fused_post_body<FT>(qs[blockIdx.x], freeze, sh);
}

// The four per-QP phases between the factor and the evaluation in ONE
// workgroup per QP: predictor solve, the middle phase (k_fused_mid), corrector
// solve, the corrector back-substitution and update (k_fused_post) -- no
// dependency crosses QPs, so a QP moves on when its own phase is done instead
// of waiting for the whole batch at three kernel boundaries.  Each phase is
// the kernel's code (trsv_small.h, the bodies above) with a workgroup
// barrier in between (its global stores visible to the next phase's loads:
// every wave of the workgroup shares the CU's L1).  NW = 8: the same values
// as the separate launches, bitwise; NW = 16: the middle / post reductions
// over 16 wave partials.  (NW = 8: at most 128 VGPRs, two workgroups per CU
// like trsv_small_kernel<8>.)
template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW == 8 ? 4 : 1))) void k_fused_solves(const QPDev* __restrict__ qs, const double* __restrict__ K,
                                                          int64_t ld, int N, const double* D,
                                                          const double* __restrict__ Linv, double* b,
                                                          int64_t sK, int64_t sD, int64_t sL, int64_t sb,
                                                          int freeze) {
  // (b and D without __restrict__: the middle and post phases reach the
  // same vectors through qs[i].b / the QP's D as well)
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ double sh[NW];
  const int64_t i = blockIdx.x;
  const QPDev& q = qs[i];
  K += i * sK;
  D += i * sD;
  Linv += i * sL;
  b += i * sb;
  trsv_small_body<NW>(K, ld, N, D, Linv, b, sm);
  __syncthreads();
  fused_mid_body<64 * NW>(q, sh);
  __syncthreads();
  trsv_small_body<NW>(K, ld, N, D, Linv, b, sm);
  __syncthreads();
  fused_post_body<64 * NW>(q, freeze, sh);
}

// Evaluation of the new iterate (Qx, Ax, Cx, A^T lambda_A, C^T lambda_C,
// then residuals, f, res, mu): gridDim.x workgroups per QP (blockIdx.y)
// share the matvec rows and transpose columns; the last to arrive (counter
// q.done, reset by it) runs the residual pass and the stats.
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(8))) void k_fused_eval(const QPDev* __restrict__ qs) {
  const QPDev& q = qs[blockIdx.y];
  __shared__ double sh[FT / 64];
  __shared__ unsigned last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = q.n, m = q.m, p = q.p, N = q.N;
  const int gw = blockIdx.x * (FT / 64) + wave, nw = gridDim.x * (FT / 64);
  const double* x = q.v[X];
  const int nr = n + m + p;
  auto row_ptr = [&](int r) {
    return r < n ? q.Q + (int64_t)r * q.ldn
                 : r < n + m ? q.A + (int64_t)(r - n) * q.ldn : q.C + (int64_t)(r - n - m) * q.ldn;
  };
  // four rows per wave at a time (their loads interleaved); each row's sum
  // in row_dot's order
  for (int r0 = gw * 4; r0 < nr; r0 += nw * 4) {
    double s0[4], s1[4];
    const double* rp[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s0[k] = s1[k] = 0.0;
      rp[k] = row_ptr(r0 + k < nr ? r0 + k : r0);
    }
    int j = lane * 2;
    for (; j + 1 < n; j += 128) {
      const double2 b = *reinterpret_cast<const double2*>(x + j);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double2 a = *reinterpret_cast<const double2*>(rp[k] + j);
        s0[k] += a.x * b.x;
        s1[k] += a.y * b.y;
      }
    }
    if (j < n) {
#pragma unroll
      for (int k = 0; k < 4; ++k) s0[k] += rp[k][j] * x[j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double d = wave_sum(s0[k] + s1[k]);
      const int r = r0 + k;
      if (lane == 0 && r < nr) st_sc1(r < n ? &q.Qx[r] : r < n + m ? &q.Ax[r - n] : &q.Cx[r - n - m], d);
    }
  }
  // transposes: one thread per (column j, chunk of FCH rows), the chunk
  // summed in row order (its loads all in flight), the chunk partials then
  // added in chunk order through LDS; passes of FT / nch columns spread over
  // the QP's workgroups (a thread per column walking all the rows was
  // ~16 us of dependent load batches at C4)
  constexpr int FCH = 8;
  __shared__ double tp[FT];
  auto transpose = [&](const double* M, auto yf, int rows, double* out) {
    const int nch = (rows + FCH - 1) / FCH;
    if (nch > FT) {  // (not at the fused path's sizes) thread per column
      for (int j = blockIdx.x * FT + tid; j < n; j += gridDim.x * FT) {
        double tot = 0.0;
        for (int i0 = 0; i0 < rows; i0 += FCH) {
          const int i1 = i0 + FCH < rows ? i0 + FCH : rows;
          double c = 0.0;
          for (int i = i0; i < i1; ++i) c += M[(int64_t)i * q.ldn + j] * yf(i);
          tot += c;
        }
        st_sc1(&out[j], tot);
      }
      return;
    }
    const int cpp = FT / nch;  // columns per pass
    const int jj = tid % cpp, h = tid / cpp;
    const int npass = (n + cpp - 1) / cpp;
    for (int pi = blockIdx.x; pi < npass; pi += gridDim.x) {  // (uniform per workgroup)
      const int j = pi * cpp + jj;
      double c = 0.0;
      if (h < nch && j < n) {
        const int i0 = h * FCH, i1 = i0 + FCH < rows ? i0 + FCH : rows;
#pragma unroll
        for (int i = i0; i < i0 + FCH; ++i)
          if (i < i1) c += M[(int64_t)i * q.ldn + j] * yf(i);
      }
      __syncthreads();  // the previous pass's reads of tp
      tp[tid] = c;
      __syncthreads();
      if (tid < cpp && j < n) {
        double tot = 0.0;
        for (int k = 0; k < nch; ++k) tot += tp[k * cpp + tid];
        st_sc1(&out[j], tot);
      }
    }
  };
  if (m) transpose(q.A, [&](int i) { return a_dual(q, i); }, m, q.ATl);
  if (p) transpose(q.C, [&](int i) { return q.v[LC][i]; }, p, q.CTl);
  // arrival (sync.h protocol: write-through data, vmcnt drained, barrier, one
  // agent-scope atomic); no cache-wide fences
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(q.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!last) return;
  if (tid == 0) st_sc1(q.done, 0u);
  double res2 = 0.0, comp = 0.0, fa = 0.0, fb = 0.0;
  for (int t = tid; t < N; t += FT) residual_elem<true>(q, t, 0.0, res2, comp, fa, fb);
  res2 = block_allsum<FT>(res2, sh);
  comp = block_allsum<FT>(comp, sh);
  fa = block_allsum<FT>(fa, sh);
  fb = block_allsum<FT>(fb, sh);
  if (tid == 0) {
    const double res = sqrt(res2);
    const int cnt = comp_count(q);
    const double mu = cnt == 0 ? 0.0 : comp / (double)cnt;
    q.scal[SC_F] = fa + fb;
    q.scal[SC_RES] = res;
    q.scal[SC_MU] = mu;
    q.scal[SC_CONVERGED] = (res < 1e-8 && mu < 1e-8) ? 1.0 : 0.0;  // Optimizer.cpp:124,133
  }
}

// about two workgroups per CU: a lone workgroup per QP cannot keep enough
// loads in flight
static int fused_split(int B) {
  const int s = (2 * device_cus() + B - 1) / B;
  return s < 1 ? 1 : (s > 8 ? 8 : s);
}

hipError_t qp_fused_pre(const QPBatch& qb, int restart, int* info, hipStream_t st, int kmode) {
  if (kmode != KMODE_K && !qb.h.K0) return hipErrorInvalidValue;
  // the diagonal-only mode has no copy to spread: one workgroup per QP
  const int split = kmode == KMODE_K0_DIAG ? 1 : fused_split(qb.B);
  hipLaunchKernelGGL(k_fused_pre, dim3(split, qb.B), dim3(FT), 0, st, qb.d, kmode == KMODE_K0_OFFDIAG ? 0 : restart,
                     kmode == KMODE_K0_OFFDIAG ? nullptr : info, kmode);
  return hipGetLastError();
}
hipError_t qp_fused_mid(const QPBatch& qb, hipStream_t st) {
  hipLaunchKernelGGL(k_fused_mid, dim3(qb.B), dim3(FT), 0, st, qb.d);
  return hipGetLastError();
}
hipError_t qp_fused_solves(const QPBatch& qb, const double* K, int64_t ld, int N, const double* D, const double* Linv,
                           double* b, int64_t sK, int64_t sD, int64_t sL, int64_t sb, int freeze, hipStream_t st) {
  if (!fused_solves_ok(N, ld)) return hipErrorInvalidValue;
  // 16 waves when the batch leaves a CU per QP, 8 when QPs share CUs (trsv.hip)
  if (qb.B <= device_cus())
    hipLaunchKernelGGL(k_fused_solves<16>, dim3(qb.B), dim3(64 * 16), trsv_small_lds(N, 16), st, qb.d, K, ld, N, D,
                       Linv, b, sK, sD, sL, sb, freeze);
  else
    hipLaunchKernelGGL(k_fused_solves<8>, dim3(qb.B), dim3(64 * 8), trsv_small_lds(N, 8), st, qb.d, K, ld, N, D, Linv,
                       b, sK, sD, sL, sb, freeze);
  return hipGetLastError();
}
// the evaluation's workgroups per QP: enough for two row passes (4 rows per
// wave, 8 waves) as long as the whole grid stays resident (8 waves per SIMD
// at 64 VGPRs: 4 workgroups per CU).  C4: B = 1024 -> 1, B = 128 -> 5
// (0.038 -> 0.035 ms against the 4 of fused_split; 2 or 8 slower,
// profiles/r05_s/c4_eval_split_ab.txt)
static int eval_split(const QPBatch& qb) {
  const int cap = 4 * device_cus() / qb.B;
  const int rows = (qb.h.n + qb.h.m + qb.h.p + 63) / 64;
  const int s = rows < cap ? rows : cap;
  return s < 1 ? 1 : (s > 8 ? 8 : s);
}
hipError_t qp_fused_eval(const QPBatch& qb, hipStream_t st) {
  hipLaunchKernelGGL(k_fused_eval, dim3(eval_split(qb), qb.B), dim3(FT), 0, st, qb.d);
  return hipGetLastError();
}
hipError_t qp_fused_post(const QPBatch& qb, int freeze, hipStream_t st) {
  hipLaunchKernelGGL(k_fused_post, dim3(qb.B), dim3(FT), 0, st, qb.d, freeze);
  hipLaunchKernelGGL(k_fused_eval, dim3(eval_split(qb), qb.B), dim3(FT), 0, st, qb.d);
  return hipGetLastError();
}

}  // namespace ipmz
