// Whole LDL^T of one small KKT matrix per workgroup (config C4: batches of
// N = 320 systems).  Replaces LinearSolvers::ldlt_decomposition
// (LinearSolvers.cpp:14-42) for the batched path: same factor (unit-lower L
// in the strict lower triangle of K, D, the 1e-8 zero-pivot rule inside
// diag64_body), blocked by 64 columns, right-looking, every step inside ONE
// workgroup -- no launch boundaries, no inter-workgroup hand-offs:
//   for each 64-column block J:
//     diag64_body: factor the diagonal block (L_JJ, D_J, L_JJ^{-1})
//     TRSM  : for every 64-row chunk c below: W_c = A[c, J] L_JJ^{-T},
//             L[c, J] = W_c / D_J                       (f64 MFMA 16x16x4)
//     update: A[c, q] -= L[c, J] W_q^T, J < q <= c      (f64 MFMA 16x16x4)
// The multi-launch batched factor paid a launch + a grid-wide drain per
// inner block and per update (and left half the chip idle at 128 QPs per
// GPU); here the only serialization is the algorithm's own.  LDS: the two
// 64 x DS operand tiles double as diag64_body's M and X (66.5 KB).  Eight
// waves (two per SIMD) split every 64 x 64 MFMA tile so one wave's LDS and
// memory waits overlap the other's MFMAs; operand tiles for the next step
// are loaded into registers while the current one computes.
#include "common.h"
#include "kernels.h"
#include "diag64.h"
#include "sync.h"

namespace ipmz {

namespace {
typedef Mfma<double> MF;
typedef MF::acc_t acc_t;

// SNW waves per workgroup (8: two per SIMD)
template <int SNW>
struct Cfg {
  static constexpr int SNT = 64 * SNW;        // threads
  static constexpr int SFR = 64 / SNW;        // tile rows fetched per thread
  static constexpr int SNN = 4 * 4 / SNW;     // 16-column MFMA blocks per wave (rows: 16 (w & 3)..)
};

// 64 x 64 tile rows [0, nrows) of a row-major source (row stride lds): wave w
// loads rows w, w+SNW, ... (one 512-byte row per load instruction); rows
// past nrows read row 0 and are zeroed on the LDS store.
template <int SNW>
__device__ __forceinline__ void tile_fetch(const double* __restrict__ src, int64_t lds, int nrows,
                                           double (&v)[Cfg<SNW>::SFR]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < Cfg<SNW>::SFR; ++i) {
    const int rr = wave + SNW * i;
    v[i] = src[(int64_t)(rr < nrows ? rr : 0) * lds + lane];
  }
}
// the same with agent-scope loads (data another workgroup of the launch wrote)
template <int SNW>
__device__ __forceinline__ void tile_fetch_sc(const double* __restrict__ src, int64_t lds, int nrows,
                                              double (&v)[Cfg<SNW>::SFR]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < Cfg<SNW>::SFR; ++i) {
    const int rr = wave + SNW * i;
    v[i] = ld_sc1(&src[(int64_t)(rr < nrows ? rr : 0) * lds + lane]);
  }
}
template <int SNW>
__device__ __forceinline__ void tile_put(double* dst, int nrows, const double (&v)[Cfg<SNW>::SFR]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < Cfg<SNW>::SFR; ++i) {
    const int rr = wave + SNW * i;
    dst[rr * DS + lane] = rr < nrows ? v[i] : 0.0;
  }
}
// this wave's part of the 64 x 64 result: rows 16 (w & 3) .. +15, column
// blocks n0 + (0 .. SNN-1), n0 = SNN (w >> 2)
__device__ __forceinline__ int tile_r0() { return 16 * ((threadIdx.x >> 6) & 3); }
template <int SNW>
__device__ __forceinline__ int tile_n0() { return Cfg<SNW>::SNN * (threadIdx.x >> 8); }
// acc[n] (+)= sgn * As[rows, :] Bs[16 (n0 + n).., :]^T.  LOWER: Bs is
// lower triangular and only its lower part is meaningful (the diagonal
// factor's L^{-1} image, left in LDS): entries k > row read as 0.
template <int SNW, bool NEG, bool LOWER = false>
__device__ __forceinline__ void tile_mma(const double* As, const double* Bs, acc_t (&acc)[Cfg<SNW>::SNN]) {
  const int lane = threadIdx.x & 63;
  const int arow = tile_r0() + (lane & 15), n0 = tile_n0<SNW>();
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (lane >> 4);
    const double a = NEG ? -As[arow * DS + k] : As[arow * DS + k];
#pragma unroll
    for (int n = 0; n < Cfg<SNW>::SNN; ++n) {
      const int brow = 16 * (n0 + n) + (lane & 15);
      const double b = Bs[brow * DS + k];
      acc[n] = MF::mma(a, LOWER ? (k <= brow ? b : 0.0) : b, acc[n]);
    }
  }
}
}  // namespace

template <int SNW>
__global__ __launch_bounds__(64 * SNW) __attribute__((amdgpu_waves_per_eu(2))) void ldlt_small_kernel(double* __restrict__ K, int64_t ld, int N,
                                                         double* __restrict__ D, double* __restrict__ Linv,
                                                         double* __restrict__ W, int* __restrict__ info, int64_t sK,
                                                         int64_t sD, int64_t sL, int64_t sW,
                                                         const double* __restrict__ K0) {
  constexpr int SFR = Cfg<SNW>::SFR, SNN = Cfg<SNW>::SNN;
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64];
  const int64_t qp = blockIdx.x;
  K += qp * sK;
  if (K0) K0 += qp * sK;  // the assembled matrix: block column 0's steps read it (first touch), L goes to K
  D += qp * sD;
  Linv += qp * sL;
  W += qp * sW;  // N x 64 row-major: the current block column's W = L D
  const int lane = threadIdx.x & 63;
  const int r0 = tile_r0(), n0 = tile_n0<SNW>();
  double* As = smem;
  double* Bs = smem + 64 * DS;
  const int nblk = (N + 63) / 64;
  auto nrows = [&](int c) { return N - 64 * c < 64 ? N - 64 * c : 64; };
  for (int J = 0; J < nblk; ++J) {
    const int J0 = 64 * J;
    const double* KS = (J == 0 && K0) ? K0 : K;  // where this step's not yet updated tiles are read
    diag64_body<false, false, double, false, SNW>(K, ld, J0, nrows(J), D, Linv + (int64_t)J * 64 * 64, info, smem,
                                                  smem + 64 * DS, smem + 2 * 64 * DS, nullptr, NoHook(), KS);
    if (J == nblk - 1) break;
    __syncthreads();  // diag64_body's L, D, L^{-1} stores are visible to the workgroup
    // ---- TRSM of the chunks below (block J is full: J0 + 64 < N), with
    // L_JJ^{-1} and the pivots straight from diag64_body's LDS images (X in
    // Bs, lower part; dsh) -- no global round trip on the chain
    double v[SFR], u[SFR];
    tile_fetch<SNW>(KS + (int64_t)(J0 + 64) * ld + J0, ld, nrows(J + 1), v);
    const double* dsh = smem + 2 * 64 * DS;
    double rd[SNN];
#pragma unroll
    for (int n = 0; n < SNN; ++n) rd[n] = 1.0 / dsh[16 * (n0 + n) + (lane & 15)];
    for (int c = J + 1; c < nblk; ++c) {
      const int rows = nrows(c);
      tile_put<SNW>(As, rows, v);
      __syncthreads();
      if (c + 1 < nblk) tile_fetch<SNW>(KS + (int64_t)(64 * (c + 1)) * ld + J0, ld, nrows(c + 1), v);
      acc_t acc[SNN];
#pragma unroll
      for (int n = 0; n < SNN; ++n) acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
      tile_mma<SNW, false, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows) {
            W[(int64_t)(64 * c + row) * 64 + col] = acc[n][g];
            K[(int64_t)(64 * c + row) * ld + J0 + col] = acc[n][g] * rd[n];
          }
        }
      }
      __syncthreads();  // As / Bs reads done before the next tile is staged
    }
    // ---- trailing update of the lower triangle below block J, tile (c, q)
    // in row order (the next diagonal block first); L[c, J] staged once per
    // row of tiles
    int c = J + 1, q = J + 1;
    tile_fetch<SNW>(K + (int64_t)(64 * c) * ld + J0, ld, nrows(c), v);  // L[c, J]
    tile_fetch<SNW>(W + (int64_t)(64 * q) * 64, 64, nrows(q), u);       // W_q
    for (;;) {
      const int rows = nrows(c);
      if (q == J + 1) tile_put<SNW>(As, rows, v);
      tile_put<SNW>(Bs, nrows(q), u);
      // the target tile C: its loads stay in flight through the MFMA chain,
      // which accumulates -L W^T from zero; C is added at the end
      acc_t acc[SNN], cv[SNN];
      const bool diag = q == c;
      // this lane's elements: rows r0 + (lane >> 4) + 4g, columns 16 (n0 + n) + (lane & 15)
      const int64_t toff = (int64_t)(64 * c + r0 + (lane >> 4)) * ld + 64 * q + 16 * n0 + (lane & 15);
      double* Ct = K + toff;
      const double* Cs = KS + toff;  // (block column 0's step: the assembled matrix)
      const double* Ct0 = KS + (int64_t)(64 * c) * ld + 64 * q;
      const int64_t ld4 = 4 * ld;
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
        acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          const bool in = row < rows && (!diag || col <= row);
          cv[n][g] = *(in ? Cs + g * ld4 + 16 * n : Ct0);  // (out-of-tile lanes: a valid dummy address)
        }
      }
      __syncthreads();
      // next tile's operands
      int cn = c, qn = q + 1;
      if (qn > cn) {
        ++cn;
        qn = J + 1;
      }
      const bool more = cn < nblk;
      if (more) {
        if (qn == J + 1) tile_fetch<SNW>(K + (int64_t)(64 * cn) * ld + J0, ld, nrows(cn), v);
        tile_fetch<SNW>(W + (int64_t)(64 * qn) * 64, 64, nrows(qn), u);
      }
      tile_mma<SNW, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows && (!diag || col <= row)) Ct[g * ld4 + 16 * n] = cv[n][g] + acc[n][g];
        }
      }
      __syncthreads();  // As / Bs free; the tile's stores visible to the next diagonal factor
      if (!more) break;
      c = cn;
      q = qn;
    }
  }
}

// ---------------------------------------------------------------------------
// The same factor with TWO workgroups per QP, for batches that leave CUs
// idle (2B <= #CU: C4's 128 QPs per GPU at 8 GPUs; N = 320, B = 128: 194 ->
// 177 us -- the five 64-column diagonal blocks, ~15 us each, stay on one
// chain).  Role 0 carries the
// critical path -- the diagonal block J, the TRSM of every chunk below it and
// the trailing tiles of column J+1 (which hold the next diagonal block and
// the next TRSM's operands) -- and role 1, on another CU, the rest of the
// trailing update of step J (columns J+2..), in the shadow of role 0's next
// diagonal factor.  Hand-offs per step (sync.h protocol: write-through
// stores, vmcnt drain, barrier, one flag store; consumers poll and read with
// agent-scope loads):
//   LW[J]    role 0 -> 1: L(c, J) in K and W(c, J) (parity J & 1 of the
//            two W buffers) for every chunk c > J
//   DONE[J]  role 1 -> 0: step J's tiles of columns >= J+2 stored (role 0
//            needs column J+2 of them at step J+1)
// Each element keeps the single-workgroup kernel's arithmetic (the same MFMA
// tiles in the same order), so the factor is identical to it.
template <int SNW>
__global__ __launch_bounds__(64 * SNW) void ldlt_small_pair_kernel(double* __restrict__ K, int64_t ld, int N,
                                                              double* __restrict__ D, double* __restrict__ Linv,
                                                              double* __restrict__ W, int* __restrict__ info,
                                                              int64_t sK, int64_t sD, int64_t sL, int64_t sW,
                                                              unsigned* __restrict__ flags, unsigned* __restrict__ err,
                                                              const double* __restrict__ K0) {
  constexpr int SFR = Cfg<SNW>::SFR, SNN = Cfg<SNW>::SNN;
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64];
  __shared__ unsigned sh_ok;
  const int64_t qp = blockIdx.x >> 1;
  const int role = blockIdx.x & 1;
  K += qp * sK;
  if (K0) K0 += qp * sK;  // block column 0's steps read the assembled matrix (not written by this launch)
  D += qp * sD;
  Linv += qp * sL;
  W += qp * sW;  // two N x 64 row-major buffers (parity of J): W = L D of block column J
  unsigned* LW = flags + qp * IPMZ_PAIR_FLAGS;
  unsigned* DONE = LW + IPMZ_PAIR_FLAGS / 2;
  const int lane = threadIdx.x & 63;
  const int r0 = tile_r0(), n0 = tile_n0<SNW>();
  double* As = smem;
  double* Bs = smem + 64 * DS;
  const int nblk = (N + 63) / 64;
  auto nrows = [&](int c) { return N - 64 * c < 64 ? N - 64 * c : 64; };
  auto Wj = [&](int J) { return W + (int64_t)(J & 1) * N * 64; };
  // tiles (c, q), c >= q, for q in [qlo, qhi], in row order, -= L(c, J) W_q^T;
  // operands of the next tile loaded while the current one computes.  All
  // global traffic agent-scope: L / W come from role 0, tiles of column J+2
  // go to it.
  auto trail = [&](int J, int qlo, int qhi) {
    if (qlo > qhi || qlo >= nblk) return;
    const double* Wb = Wj(J);
    double v[SFR], u[SFR];
    int c = qlo, q = qlo;
    tile_fetch_sc<SNW>(K + (int64_t)(64 * c) * ld + 64 * J, ld, nrows(c), v);  // L[c, J]
    tile_fetch_sc<SNW>(Wb + (int64_t)(64 * q) * 64, 64, nrows(q), u);           // W_q
    for (;;) {
      const int rows = nrows(c);
      if (q == qlo) tile_put<SNW>(As, rows, v);
      tile_put<SNW>(Bs, nrows(q), u);
      acc_t acc[SNN], cv[SNN];
      const bool diag = q == c;
      const int64_t toff = (int64_t)(64 * c + r0 + (lane >> 4)) * ld + 64 * q + 16 * n0 + (lane & 15);
      double* Ct = K + toff;
      const double* Cs = ((J == 0 && K0) ? K0 : K) + toff;  // block column 0's step: the assembled matrix
      const double* Ct0 = K + (int64_t)(64 * c) * ld + 64 * q;
      const int64_t ld4 = 4 * ld;
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
        acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          const bool in = row < rows && (!diag || col <= row);
          cv[n][g] = ld_sc1(in ? Cs + g * ld4 + 16 * n : Ct0);
        }
      }
      __syncthreads();
      int cn = c, qn = q + 1;
      if (qn > cn || qn > qhi) {
        ++cn;
        qn = qlo;
      }
      const bool more = cn < nblk;
      if (more) {
        if (qn == qlo) tile_fetch_sc<SNW>(K + (int64_t)(64 * cn) * ld + 64 * J, ld, nrows(cn), v);
        tile_fetch_sc<SNW>(Wb + (int64_t)(64 * qn) * 64, 64, nrows(qn), u);
      }
      tile_mma<SNW, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows && (!diag || col <= row)) st_sc1(Ct + g * ld4 + 16 * n, cv[n][g] + acc[n][g]);
        }
      }
      __syncthreads();
      if (!more) break;
      c = cn;
      q = qn;
    }
  };
  if (role == 1) {
    for (int J = 0; J + 2 < nblk; ++J) {
      if (!wait_flag(&LW[J], err, &sh_ok)) return;
      trail(J, J + 2, nblk - 1);
      publish(&DONE[J]);
    }
    return;
  }
  for (int J = 0; J < nblk; ++J) {
    const int J0 = 64 * J;
    const double* KS = (J == 0 && K0) ? K0 : K;  // where this step's not yet updated tiles are read
    // block J was last updated by this workgroup (column J+1 of step J-1) or
    // before the DONE[J-2] wait of step J-1 (agent-scope loads: LSC)
    diag64_body<false, true, double, false, SNW>(K, ld, J0, nrows(J), D, Linv + (int64_t)J * 64 * 64, info, smem,
                                                 smem + 64 * DS, smem + 2 * 64 * DS, nullptr, NoHook(), KS);
    if (J == nblk - 1) break;
    __syncthreads();
    // ---- TRSM of every chunk below, published for role 1
    double v[SFR];
    tile_fetch_sc<SNW>(KS + (int64_t)(J0 + 64) * ld + J0, ld, nrows(J + 1), v);
    const double* dsh = smem + 2 * 64 * DS;
    double* Wb = Wj(J);
    double rd[SNN];
#pragma unroll
    for (int n = 0; n < SNN; ++n) rd[n] = 1.0 / dsh[16 * (n0 + n) + (lane & 15)];
    for (int c = J + 1; c < nblk; ++c) {
      const int rows = nrows(c);
      tile_put<SNW>(As, rows, v);
      __syncthreads();
      if (c + 1 < nblk) tile_fetch_sc<SNW>(KS + (int64_t)(64 * (c + 1)) * ld + J0, ld, nrows(c + 1), v);
      acc_t acc[SNN];
#pragma unroll
      for (int n = 0; n < SNN; ++n) acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
      tile_mma<SNW, false, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows) {
            st_sc1(&Wb[(int64_t)(64 * c + row) * 64 + col], acc[n][g]);
            st_sc1(&K[(int64_t)(64 * c + row) * ld + J0 + col], acc[n][g] * rd[n]);
          }
        }
      }
      __syncthreads();
    }
    publish(&LW[J]);
    // ---- column J+1 of the trailing update (the next diagonal block and the
    // next TRSM's operands), after role 1's step J-1 (it updated column J+1)
    if (J >= 1 && !wait_flag(&DONE[J - 1], err, &sh_ok)) return;
    trail(J, J + 1, J + 1);
  }
}

// 2B workgroups must all be resident at once to help: 256 VGPRs per lane x 8
// waves fill a CU, so one workgroup per CU -- 2B <= #CU (B = 128 at 8 GPUs)
bool small_pair_eligible(int B, int N) { return 2 * B <= device_cus() && N > 64 && N <= IPMZ_SMALL_NMAX; }

hipError_t ldlt_factor_small_batched(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int* info,
                                     hipStream_t st, const BatchStrides& bs) {
  if (N <= 0 || bs.B <= 0) return hipSuccess;
  // a batch that leaves CUs idle: two workgroups per QP (flags zeroed here)
  if (bs.pflags && small_pair_eligible(bs.B, N)) {
    hipError_t e = hipMemsetAsync(bs.pflags, 0, ((size_t)bs.B * IPMZ_PAIR_FLAGS + 1) * sizeof(unsigned), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ldlt_small_pair_kernel<8>, dim3(2 * bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, W, info,
                       bs.sK, bs.sD, bs.sL, bs.sW, bs.pflags, bs.pflags + (size_t)bs.B * IPMZ_PAIR_FLAGS, bs.K0);
    return hipGetLastError();
  }
  // 8 waves (two per SIMD) also when the batch leaves a CU per QP: 16 waves
  // measured slower (N = 320, B = 128: 249 vs 190 us)
  hipLaunchKernelGGL(ldlt_small_kernel<8>, dim3(bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, W, info, bs.sK, bs.sD,
                     bs.sL, bs.sW, bs.K0);
  return hipGetLastError();
}

// experiment entry (tools/kbench.cpp "smallv"): the one-workgroup factor with
// SNW = 4 waves (two workgroups -- two QPs -- per CU) or 8
hipError_t ldlt_factor_small_variant(int snw, double* K, int64_t ld, int N, double* D, double* Linv, double* W,
                                     int* info, hipStream_t st, const BatchStrides& bs) {
  if (snw == 4)
    hipLaunchKernelGGL(ldlt_small_kernel<4>, dim3(bs.B), dim3(64 * 4), 0, st, K, ld, N, D, Linv, W, info, bs.sK,
                       bs.sD, bs.sL, bs.sW, bs.K0);
  else
    hipLaunchKernelGGL(ldlt_small_kernel<8>, dim3(bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, W, info, bs.sK,
                       bs.sD, bs.sL, bs.sW, bs.K0);
  return hipGetLastError();
}

}  // namespace ipmz
