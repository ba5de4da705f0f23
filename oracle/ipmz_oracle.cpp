// ipmz_oracle -- CPU restatement of ipm-zoo's numerical interior-point Newton
// step (albfre/ipm-zoo @ 2025-07-04, /root/reference).
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg load this library, and only as the checker or
// the timed CPU baseline -- never as the product path.  The product
// (ipm-zoo_amd/, libipmz.so) never links it and has no CPU fallback.
//
// Pinned by the golden vectors that tests/golden/make_golden.py generates
// from the compiled reference (oracle/Makefile.ref + oracle/ref_harness.cpp):
// LDL^T factor/solve and the SlackedSlacks Newton iterations compare BITWISE
// (tests/test_oracle_golden.py).  The Regularization-equality formulation
// (config C3) has no end-to-end reference (the reference asserts on its
// scalar block, Evaluation.cpp:57-60): its KKT / factor / solve are pinned at
// component level, its rhs and back-substitution formulas are the reference's
// own symbolic output (tests/golden/formulations.txt).
//
// Build: g++ -O3 -ffp-contract=off -fPIC -shared (no -march=native: FMA
// contraction changes the rounding).  Every expression below
// keeps the reference evaluator's operand order (Evaluation.cpp:102-176):
// Sum terms are added left to right, a - b is a + (-b) (bit-identical),
// Product terms are multiplied left to right, X^{-1} is an element-wise
// reciprocal with 0 -> sqrt(DBL_MAX) (Evaluation.cpp:267-271).
#include <chrono>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace {

using Vec = std::vector<double>;

// ---------------------------------------------------------------------------
// Synthetic QP generator.  Identical bit-for-bit to the GPU
// in-place generator ipm-zoo_amd/csrc/qpgen.h and to oracle/ref_harness.cpp.
inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
inline double u01(uint64_t seed, uint64_t tag, uint64_t i, uint64_t j) {
  const uint64_t key = seed ^ (tag << 56) ^ ((i << 32) + j);
  return (double)(splitmix64(key) >> 11) * 0x1.0p-53;
}
enum : uint64_t { TAG_Q = 1, TAG_C = 2, TAG_A = 3, TAG_C_EQ = 4, TAG_D = 5 };

// Evaluation.cpp:267-271
inline double inv(double x) { return x == 0.0 ? std::sqrt(std::numeric_limits<double>::max()) : 1.0 / x; }

// Canonical Newton-variable slots.  The reference's Newton variable order
// (SymbolicOptimization get_newton_system; tests/golden/formulations.txt) is
// this order with absent blocks dropped.
enum Slot { X, LA, LC, S, P, LG, LH, LY, LZ, G, H, Y, Z, NSLOT };

struct QP {
  int64_t n, m, p;
  double delta;  // EnvironmentBuilder.cpp:48
  // EqualityHandling::None (tests/golden/formulations.txt): no p, a zero
  // (lambda_C, lambda_C) block -- the reference's "indefinite" case, factored
  // with Bunch-Kaufman (Optimizer.cpp:63-75; solve_indefinite_ is ASSERT(false)
  // there, this is the completion §8f row f3 asks for)
  bool eq_none = false;
  // EqualityHandling::PenaltyFunction (formulations.txt): no p, a -mu
  // (lambda_C, lambda_C) block (mu = the environment's mu when the KKT matrix
  // is assembled), r_lambda_C := -(d + (mu*lambda_C) - (C*x)); LDL^T.  The
  // reference's evaluator asserts on the scalar block (Evaluation.cpp:57-60);
  // here it is mu * I (§8f row f4)
  bool eq_pen = false;
  // Settings (SymbolicOptimization.h:28-64, formulations.txt): InequalityHandling
  // ::Slacks -- no nonnegative slacks g, h, y, z; the complementarity rows are
  // ((X - L_x) lambda_y - mu e), ((U_x - X) lambda_z - mu e), ((S - L_A)
  // lambda_g - mu e), ((U_A - S) lambda_h - mu e) -- and one-sided / absent
  // bounds: vlo / vup = Settings::variable_bounds has Lower / Upper, alo / aup
  // = Settings::inequalities has Lower / Upper (one of them when m > 0).
  // Defaults: SlackedSlacks, Bounds::Both.
  bool slacks = false;
  bool vlo = true, vup = true, alo = true, aup = true;
  // InequalityHandling::NaiveSlacks (formulations.txt): no s and no lambda_A;
  // l_A + g = A x and A x + h = u_A with their own duals lambda_g, lambda_h,
  // which become KKT rows: the augmented system is [x, lambda_g, lambda_h,
  // lambda_C] (n + 2m + p).  The reference's evaluator asserts on its zero
  // (lambda_g, lambda_h) block (Evaluation.cpp:57-60); Bounds::Both only.
  bool naive = false;
  Vec Q, c, A, lA, uA, C, d, lx, ux;
  Vec v[NSLOT];       // iterate
  Vec daff[NSLOT], dir[NSLOT];
  double mu;          // EnvironmentBuilder.cpp:49
  int64_t size(int s) const {
    switch (s) {
      case X: return n;
      case LY: return vlo ? n : 0;
      case LZ: return vup ? n : 0;
      case Y: return vlo && !slacks ? n : 0;
      case Z: return vup && !slacks ? n : 0;
      case LA: case S: return naive ? 0 : m;
      case LG: return alo ? m : 0;
      case LH: return aup ? m : 0;
      case G: return alo && !slacks ? m : 0;
      case H: return aup && !slacks ? m : 0;
      case P: return (eq_none || eq_pen) ? 0 : p;
      default: return p;
    }
  }
  int64_t mk() const { return naive ? 2 * m : m; }  // KKT rows of the inequalities
  int64_t N() const { return n + mk() + p; }
};

// ---------------------------------------------------------------------------
// Matrix-vector products as the reference evaluates them
// (Evaluation.cpp:18-21, 35-41; Transpose materialised at :126-140, so A^T v
// is a row-dot over the transposed rows: sequential sum over the original
// row index).
void matvec(const Vec& M, int64_t rows, int64_t cols, const double* x, double* out) {
  for (int64_t i = 0; i < rows; ++i) {
    double s = 0.0;
    const double* r = M.data() + i * cols;
    for (int64_t j = 0; j < cols; ++j) s = s + r[j] * x[j];
    out[i] = s;
  }
}
void matvec_t(const Vec& M, int64_t rows, int64_t cols, const double* x, double* out) {
  for (int64_t j = 0; j < cols; ++j) {
    double s = 0.0;
    for (int64_t i = 0; i < rows; ++i) s = s + M[i * cols + j] * x[i];
    out[j] = s;
  }
}

struct Residuals {
  Vec r[NSLOT];
};

// Shorthand definitions r_v := -rhs_v (SymbolicOptimization.cpp:480-492),
// formulas: tests/golden/formulations.txt "shorthand definitions".
void residuals(const QP& q, double mu, Residuals& R) {
  const int64_t n = q.n, m = q.m, p = q.p;
  for (int s = 0; s < NSLOT; ++s) R.r[s].assign(q.size(s), 0.0);
  const Vec* v = q.v;
  Vec Qx(n), ATl(n), CTl(n), Ax(m), Cx(p);
  matvec(q.Q, n, n, v[X].data(), Qx.data());
  if (m && q.naive) {  // (A^T * (lambda_h - lambda_g))
    Vec dl(m);
    for (int64_t i = 0; i < m; ++i) dl[i] = v[LH][i] + (-v[LG][i]);
    matvec_t(q.A, m, n, dl.data(), ATl.data());
    matvec(q.A, m, n, v[X].data(), Ax.data());
  } else if (m) {
    matvec_t(q.A, m, n, v[LA].data(), ATl.data());
    matvec(q.A, m, n, v[X].data(), Ax.data());
  }
  if (p) { matvec_t(q.C, p, n, v[LC].data(), CTl.data()); matvec(q.C, p, n, v[X].data(), Cx.data()); }
  for (int64_t i = 0; i < n; ++i) {
    // r_x := (c [+ lambda_z] + (Q*x) [+ (A^T*lambda_A)] [+ (C^T*lambda_C)] [- lambda_y])
    double t = q.c[i];
    if (q.vup) t = t + v[LZ][i];
    t = t + Qx[i];
    if (m) t = t + ATl[i];
    if (p) t = t + CTl[i];
    R.r[X][i] = q.vlo ? t + (-v[LY][i]) : t;
    if (q.slacks) {
      if (q.vlo) R.r[LY][i] = ((v[X][i] + (-q.lx[i])) * v[LY][i]) + (-(mu * 1.0));  // (((X - L_x)*lambda_y) - (mu*e_x))
      if (q.vup) R.r[LZ][i] = ((q.ux[i] + (-v[X][i])) * v[LZ][i]) + (-(mu * 1.0));  // (((U_x - X)*lambda_z) - (mu*e_x))
    } else {
      if (q.vlo) {
        R.r[LY][i] = (q.lx[i] + v[Y][i]) + (-v[X][i]);  // (l_x + y - x)
        R.r[Y][i] = v[Y][i] * v[LY][i] + (-(mu * 1.0));  // ((Y*lambda_y) - (mu*e_x))
      }
      if (q.vup) {
        R.r[LZ][i] = (v[X][i] + v[Z][i]) + (-q.ux[i]);  // (x + z - u_x)
        R.r[Z][i] = v[Z][i] * v[LZ][i] + (-(mu * 1.0));
      }
    }
  }
  for (int64_t i = 0; i < m && q.naive; ++i) {
    R.r[LG][i] = (q.lA[i] + v[G][i]) + (-Ax[i]);        // (l_A + g - (A*x))
    R.r[LH][i] = (v[H][i] + Ax[i]) + (-q.uA[i]);        // (h + (A*x) - u_A)
    R.r[G][i] = v[G][i] * v[LG][i] + (-(mu * 1.0));     // ((G*lambda_g) - (mu*e_A))
    R.r[H][i] = v[H][i] * v[LH][i] + (-(mu * 1.0));
  }
  for (int64_t i = 0; i < m && !q.naive; ++i) {
    R.r[LA][i] = Ax[i] + (-v[S][i]);  // ((A*x) - s)
    if (q.alo && q.aup) R.r[S][i] = -((v[LA][i] + v[LG][i]) + (-v[LH][i]));  // -(lambda_A + lambda_g - lambda_h)
    else if (q.alo) R.r[S][i] = -(v[LA][i] + v[LG][i]);                      // -(lambda_A + lambda_g)
    else R.r[S][i] = v[LH][i] + (-v[LA][i]);                                 // (lambda_h - lambda_A)
    if (q.slacks) {
      R.r[LG][i] = ((v[S][i] + (-q.lA[i])) * v[LG][i]) + (-(mu * 1.0));  // (((S - L_A)*lambda_g) - (mu*e_A))
      R.r[LH][i] = ((q.uA[i] + (-v[S][i])) * v[LH][i]) + (-(mu * 1.0));  // (((U_A - S)*lambda_h) - (mu*e_A))
    } else {
      if (q.alo) {
        R.r[LG][i] = (q.lA[i] + v[G][i]) + (-v[S][i]);  // (l_A + g - s)
        R.r[G][i] = v[G][i] * v[LG][i] + (-(mu * 1.0));
      }
      if (q.aup) {
        R.r[LH][i] = (v[H][i] + v[S][i]) + (-q.uA[i]);  // (h + s - u_A)
        R.r[H][i] = v[H][i] * v[LH][i] + (-(mu * 1.0));
      }
    }
  }
  for (int64_t i = 0; i < p && q.eq_none; ++i) R.r[LC][i] = Cx[i] + (-q.d[i]);  // ((C*x) - d)
  for (int64_t i = 0; i < p && q.eq_pen; ++i)                                    // -(d + (mu*lambda_C) - (C*x))
    R.r[LC][i] = -((q.d[i] + mu * v[LC][i]) + (-Cx[i]));
  for (int64_t i = 0; i < p && !q.eq_none && !q.eq_pen; ++i) {
    R.r[LC][i] = (Cx[i] + q.delta * v[P][i]) + (-q.d[i]);          // ((C*x) + (delta*p) - d)
    R.r[P][i] = v[P][i] + q.delta * v[LC][i];                      // (p + (delta*lambda_C))
  }
}

// The rows that carry e and mu (get_mu_'s filter, Optimizer.cpp:250-268), in
// Newton order: g, h, y, z (SlackedSlacks) or lambda_g, lambda_h, lambda_y,
// lambda_z (Slacks).
inline void comp_rows(const QP& q, int out[4]) {
  const int ss[4] = {G, H, Y, Z}, sl[4] = {LG, LH, LY, LZ};
  for (int k = 0; k < 4; ++k) out[k] = q.slacks ? sl[k] : ss[k];
}

// Newton-variable order of the reference (absent blocks dropped).
std::vector<int> order(const QP& q) {
  std::vector<int> o;
  static const int naive_order[NSLOT] = {X, LG, LH, LC, P, LY, LZ, G, H, Y, Z, LA, S};
  for (int k = 0; k < NSLOT; ++k) {
    const int s = q.naive ? naive_order[k] : k;
    if (q.size(s) > 0) o.push_back(s);
  }
  return o;
}

// get_residual_norm_ (Optimizer.cpp:240-247): ||full rhs at mu=0||_2,
// concatenated in Newton-variable order, inner_product from 0.0.
double residual_norm(const QP& q) {
  Residuals R;
  residuals(q, 0.0, R);
  double s = 0.0;
  for (int slot : order(q))
    for (double r : R.r[slot]) {
      const double b = -r;
      s = s + b * b;
    }
  return std::sqrt(s);
}

// get_mu_ (Optimizer.cpp:249-268): mean |complementarity| at mu=0 over the
// rows containing e and mu, in Newton order (g, h, y, z).
// A complementarity row at mu (the residuals() expressions of those rows).
inline double comp_value(const QP& q, int slot, int64_t i, double mu) {
  const Vec* v = q.v;
  switch (slot) {
    case G: return v[G][i] * v[LG][i] + (-(mu * 1.0));
    case H: return v[H][i] * v[LH][i] + (-(mu * 1.0));
    case Y: return v[Y][i] * v[LY][i] + (-(mu * 1.0));
    case Z: return v[Z][i] * v[LZ][i] + (-(mu * 1.0));
    case LG: return ((v[S][i] + (-q.lA[i])) * v[LG][i]) + (-(mu * 1.0));
    case LH: return ((q.uA[i] + (-v[S][i])) * v[LH][i]) + (-(mu * 1.0));
    case LY: return ((v[X][i] + (-q.lx[i])) * v[LY][i]) + (-(mu * 1.0));
    default: return ((q.ux[i] + (-v[X][i])) * v[LZ][i]) + (-(mu * 1.0));  // LZ
  }
}

double mu_of(const QP& q) {
  int comp[4];
  comp_rows(q, comp);
  double s = 0.0;
  int64_t cnt = 0;
  for (int k = 0; k < 4; ++k) {
    const int64_t len = q.size(comp[k]);
    for (int64_t i = 0; i < len; ++i) s = s + std::abs(-comp_value(q, comp[k], i, 0.0));
    cnt += len;
  }
  return cnt == 0 ? 0.0 : s / (double)cnt;
}

// Objective 0.5 x^T Q x + c^T x (Optimizer.cpp:45-48; Product evaluation with
// the "unhandled" x^T, Evaluation.cpp:154-172).
double objective(const QP& q) {
  const int64_t n = q.n;
  Vec Qx(n);
  matvec(q.Q, n, n, q.v[X].data(), Qx.data());
  double a = 0.0, b = 0.0;
  for (int64_t i = 0; i < n; ++i) a = a + (0.5 * q.v[X][i]) * Qx[i];
  for (int64_t i = 0; i < n; ++i) b = b + q.c[i] * q.v[X][i];
  return a + b;
}

// Diagonal of the (lambda_A, lambda_A) block before negation:
// ((G^{-1}*Lambda_g) + (H^{-1}*Lambda_h))^{-1}.
inline double ds_inv(const QP& q, int64_t i) {
  return inv(inv(q.v[G][i]) * q.v[LG][i] + inv(q.v[H][i]) * q.v[LH][i]);
}
// Slacks: (((U_A - S)^{-1}*Lambda_h) + ((S - L_A)^{-1}*Lambda_g))^{-1}
inline double ds_inv_sl(const QP& q, int64_t i) {
  return inv(inv(q.uA[i] + (-q.v[S][i])) * q.v[LH][i] + inv(q.v[S][i] + (-q.lA[i])) * q.v[LG][i]);
}
// the (x, x) diagonal term added to Q_ii and the (lambda_A, lambda_A) diagonal
inline double kkt_xx(const QP& q, int64_t i, double qii) {
  const Vec* v = q.v;
  if (q.slacks) {  // (Q + ((U_x - X)^{-1}*Lambda_z) + ((X - L_x)^{-1}*Lambda_y))
    double h = qii;
    if (q.vup) h = h + inv(q.ux[i] + (-v[X][i])) * v[LZ][i];
    if (q.vlo) h = h + inv(v[X][i] + (-q.lx[i])) * v[LY][i];
    return h;
  }
  double h = qii;  // (Q [+ (Y^{-1}*Lambda_y)] [+ (Z^{-1}*Lambda_z)])
  if (q.vlo) h = h + inv(v[Y][i]) * v[LY][i];
  if (q.vup) h = h + inv(v[Z][i]) * v[LZ][i];
  return h;
}
inline double kkt_aa(const QP& q, int64_t i) {
  if (q.slacks) return -ds_inv_sl(q, i);
  if (q.alo && q.aup) return -ds_inv(q, i);                   // -((G^{-1}*Lambda_g) + (H^{-1}*Lambda_h))^{-1}
  if (q.alo) return -(inv(q.v[LG][i]) * q.v[G][i]);           // -(Lambda_g^{-1}*G)
  return -(inv(q.v[LH][i]) * q.v[H][i]);                      // -(Lambda_h^{-1}*H)
}

// Augmented KKT (get_as_matrix_, Optimizer.cpp:387-391 / 441-501), dense
// row-major N x N, both triangles.
void assemble(const QP& q, double* K) {
  const int64_t n = q.n, m = q.m, p = q.p, N = q.N();
  std::memset(K, 0, sizeof(double) * (size_t)(N * N));
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t j = 0; j < n; ++j) K[i * N + j] = q.Q[i * n + j];
    K[i * N + i] = kkt_xx(q, i, q.Q[i * n + i]);  // elementwise_diag_mat_op
  }
  for (int64_t r = 0; r < m && q.naive; ++r) {  // | -A | -(L_g^{-1}*G) | 0 |, | A | 0 | -(L_h^{-1}*H) |
    for (int64_t j = 0; j < n; ++j) {
      K[(n + r) * N + j] = -q.A[r * n + j];
      K[j * N + n + r] = -q.A[r * n + j];
      K[(n + m + r) * N + j] = q.A[r * n + j];
      K[j * N + n + m + r] = q.A[r * n + j];
    }
    K[(n + r) * N + n + r] = -(inv(q.v[LG][r]) * q.v[G][r]);
    K[(n + m + r) * N + n + m + r] = -(inv(q.v[LH][r]) * q.v[H][r]);
  }
  for (int64_t r = 0; r < m && !q.naive; ++r) {
    for (int64_t j = 0; j < n; ++j) {
      K[(n + r) * N + j] = q.A[r * n + j];
      K[j * N + n + r] = q.A[r * n + j];
    }
    K[(n + r) * N + n + r] = kkt_aa(q, r);
  }
  const int64_t c0 = n + q.mk();
  for (int64_t r = 0; r < p; ++r) {
    for (int64_t j = 0; j < n; ++j) {
      K[(c0 + r) * N + j] = q.C[r * n + j];
      K[j * N + c0 + r] = q.C[r * n + j];
    }
    K[(c0 + r) * N + c0 + r] = q.eq_none ? 0.0 : q.eq_pen ? -q.mu : -(q.delta * q.delta);
  }
}

// Augmented rhs (tests/golden/formulations.txt "augmented system rhs").
void augmented_rhs(const QP& q, const Residuals& R, double* b) {
  const int64_t n = q.n, m = q.m, p = q.p;
  const Vec* v = q.v;
  for (int64_t i = 0; i < n; ++i) {
    const double rx = R.r[X][i];
    if (q.slacks) {  // (((U_x - X)^{-1}*r_lz) - r_x - ((X - L_x)^{-1}*r_ly)), absent terms dropped
      double t = q.vup ? inv(q.ux[i] + (-v[X][i])) * R.r[LZ][i] + (-rx) : -rx;
      if (q.vlo) t = t + (-(inv(v[X][i] + (-q.lx[i])) * R.r[LY][i]));
      b[i] = t;
      continue;
    }
    const double tz = q.vup ? inv(v[Z][i]) * (R.r[Z][i] + (-(v[LZ][i] * R.r[LZ][i]))) : 0.0;
    const double ty = q.vlo ? inv(v[Y][i]) * (R.r[Y][i] + (-(v[LY][i] * R.r[LY][i]))) : 0.0;
    if (q.vlo && q.vup) b[i] = (tz + (-rx)) + (-ty);  // ((Z^{-1}*(r_z - (L_z*r_lz))) - r_x - (Y^{-1}*(...)))
    else if (q.vup) b[i] = tz + (-rx);               // ((Z^{-1}*(r_z - (L_z*r_lz))) - r_x)
    else if (q.vlo) b[i] = -(rx + ty);               // -(r_x + (Y^{-1}*(r_y - (L_y*r_ly))))
    else b[i] = -rx;                                 // -r_x
  }
  for (int64_t i = 0; i < m && q.naive; ++i) {
    b[n + i] = inv(v[LG][i]) * R.r[G][i] + (-R.r[LG][i]);      // ((L_g^{-1}*r_g) - r_lg)
    b[n + m + i] = inv(v[LH][i]) * R.r[H][i] + (-R.r[LH][i]);  // ((L_h^{-1}*r_h) - r_lh)
  }
  for (int64_t i = 0; i < m && !q.naive; ++i) {
    const double rla = R.r[LA][i], rs = R.r[S][i];
    if (q.slacks) {
      const double a = inv(q.uA[i] + (-v[S][i])) * R.r[LH][i], c = inv(v[S][i] + (-q.lA[i])) * R.r[LG][i];
      b[n + i] = ds_inv_sl(q, i) * ((a + (-rs)) + (-c)) + (-rla);
    } else if (q.alo && q.aup) {
      const double th = inv(v[H][i]) * (R.r[H][i] + (-(v[LH][i] * R.r[LH][i])));
      const double tg = inv(v[G][i]) * (R.r[G][i] + (-(v[LG][i] * R.r[LG][i])));
      b[n + i] = ds_inv(q, i) * ((th + (-rs)) + (-tg)) + (-rla);
    } else if (q.alo) {  // -(r_lA + (L_g^{-1}*(r_g + (G*r_s))) - r_lg)
      b[n + i] = -((rla + inv(v[LG][i]) * (R.r[G][i] + v[G][i] * rs)) + (-R.r[LG][i]));
    } else {  // ((L_h^{-1}*(r_h - (H*r_s))) - r_lA - r_lh)
      b[n + i] = ((inv(v[LH][i]) * (R.r[H][i] + (-(v[H][i] * rs)))) + (-rla)) + (-R.r[LH][i]);
    }
  }
  for (int64_t i = 0; i < p; ++i)  // None: -r_lambda_C ; Regularization: (delta*r_p) - r_lambda_C
    b[n + q.mk() + i] = (q.eq_none || q.eq_pen) ? -R.r[LC][i] : q.delta * R.r[P][i] + (-R.r[LC][i]);
}

// Eliminated-variable back-substitution (delta_definitions evaluated in
// reverse order, Optimizer.cpp:373-378).
void back_substitute(const QP& q, const Residuals& R, Vec* D) {
  const int64_t n = q.n, m = q.m, p = q.p;
  const Vec* v = q.v;
  for (int64_t i = 0; i < m && q.naive; ++i) {
    D[G][i] = -(inv(v[LG][i]) * (R.r[G][i] + v[G][i] * D[LG][i]));  // -(L_g^{-1}*(r_g + (G*dl_g)))
    D[H][i] = -(inv(v[LH][i]) * (R.r[H][i] + v[H][i] * D[LH][i]));
  }
  for (int64_t i = 0; i < m && !q.naive; ++i) {
    const double dla = D[LA][i], rs = R.r[S][i];
    if (q.slacks) {
      const double a = inv(q.uA[i] + (-v[S][i])) * R.r[LH][i], c = inv(v[S][i] + (-q.lA[i])) * R.r[LG][i];
      const double ds = ds_inv_sl(q, i) * (((dla + a) + (-rs)) + (-c));
      D[S][i] = ds;
      D[LG][i] = -(inv(v[S][i] + (-q.lA[i])) * (R.r[LG][i] + v[LG][i] * ds));  // -((S - L_A)^{-1}*(r_lg + (L_g*ds)))
      D[LH][i] = inv(q.uA[i] + (-v[S][i])) * (v[LH][i] * ds + (-R.r[LH][i]));  // ((U_A - S)^{-1}*((L_h*ds) - r_lh))
      continue;
    }
    double ds;
    if (q.alo && q.aup) {
      const double th = inv(v[H][i]) * (R.r[H][i] + (-(v[LH][i] * R.r[LH][i])));
      const double tg = inv(v[G][i]) * (R.r[G][i] + (-(v[LG][i] * R.r[LG][i])));
      ds = ds_inv(q, i) * ((((dla + th) + (-rs)) + (-tg)));
    } else if (q.alo) {  // (L_g^{-1}*G*(dla - r_s - (G^{-1}*(r_g - (L_g*r_lg)))))
      ds = (inv(v[LG][i]) * v[G][i]) *
           ((dla + (-rs)) + (-(inv(v[G][i]) * (R.r[G][i] + (-(v[LG][i] * R.r[LG][i]))))));
    } else {  // (L_h^{-1}*H*(dla + (H^{-1}*(r_h - (L_h*r_lh))) - r_s))
      ds = (inv(v[LH][i]) * v[H][i]) *
           ((dla + inv(v[H][i]) * (R.r[H][i] + (-(v[LH][i] * R.r[LH][i])))) + (-rs));
    }
    D[S][i] = ds;
    if (q.alo) {
      D[LG][i] = -((inv(v[G][i]) * v[LG][i]) * ((ds + inv(v[LG][i]) * R.r[G][i]) + (-R.r[LG][i])));
      D[G][i] = -(inv(v[LG][i]) * (R.r[G][i] + v[G][i] * D[LG][i]));
    }
    if (q.aup) {
      D[LH][i] = -((inv(v[H][i]) * v[LH][i]) * ((inv(v[LH][i]) * R.r[H][i] + (-R.r[LH][i])) + (-ds)));
      D[H][i] = -(inv(v[LH][i]) * (R.r[H][i] + v[H][i] * D[LH][i]));
    }
  }
  for (int64_t i = 0; i < p && !q.eq_none && !q.eq_pen; ++i) D[P][i] = -(R.r[P][i] + q.delta * D[LC][i]);
  for (int64_t i = 0; i < n; ++i) {
    const double dx = D[X][i];
    if (q.slacks) {
      if (q.vlo) D[LY][i] = -(inv(v[X][i] + (-q.lx[i])) * (R.r[LY][i] + v[LY][i] * dx));  // -((X - L_x)^{-1}*(r_ly + (L_y*dx)))
      if (q.vup) D[LZ][i] = inv(q.ux[i] + (-v[X][i])) * (v[LZ][i] * dx + (-R.r[LZ][i]));  // ((U_x - X)^{-1}*((L_z*dx) - r_lz))
      continue;
    }
    if (q.vlo) {
      D[LY][i] = -((inv(v[Y][i]) * v[LY][i]) * ((dx + inv(v[LY][i]) * R.r[Y][i]) + (-R.r[LY][i])));
      D[Y][i] = -(inv(v[LY][i]) * (R.r[Y][i] + v[Y][i] * D[LY][i]));
    }
    if (q.vup) {
      D[LZ][i] = -((inv(v[Z][i]) * v[LZ][i]) * ((inv(v[LZ][i]) * R.r[Z][i] + (-R.r[LZ][i])) + (-dx)));
      D[Z][i] = -(inv(v[LZ][i]) * (R.r[Z][i] + v[Z][i] * D[LZ][i]));
    }
  }
}

// ---------------------------------------------------------------------------
// LinearSolvers restatement (LinearSolvers.cpp:14-74), same loop and product
// order; L is a full N x N row-major matrix (zeros above, ones on diagonal).
void ldlt(int64_t n, const double* A, int64_t lda, double* L, int64_t ldl, double* D) {
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) L[i * ldl + j] = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    double sum_d = A[i * lda + i];
    const double* Li = L + i * ldl;
    for (int64_t j = 0; j < i; ++j) sum_d -= Li[j] * Li[j] * D[j];
    D[i] = sum_d == 0.0 ? 1e-8 : sum_d;  // Vanderbei zero-pivot rule, :26-28
    for (int64_t j = i + 1; j < n; ++j) {
      double sum = A[j * lda + i];
      const double* Lj = L + j * ldl;
      for (int64_t k = 0; k < i; ++k) sum -= Lj[k] * Li[k] * D[k];
      L[j * ldl + i] = sum / D[i];
    }
    L[i * ldl + i] = 1.0;
  }
}

// The same factorization, bit for bit, reorganised for large N (the C3 / C5
// parity tests run the oracle at N = 11264 / 8192 on the GPU box's host).
// Every element's running sum S[j][i] = A[j][i] - sum_k (L[j][k] * L[i][k]) *
// D[k] still subtracts its terms one at a time in increasing k with the same
// operations -- only WHEN each (j, i, k) term is applied changes:
//   for each block of nb columns [I0, I1):
//     1. the diagonal block, exactly the loop above restricted to k in [I0, i);
//     2. the rows below it (parallel over rows): k in [I0, i), then / D[i];
//     3. the trailing triangle (parallel over rows): S[j][i] -= (L[j][k] *
//        L[i][k]) * D[k] for k in [I0, I1) in order -- a right-looking update
//        whose inner loop runs over i with an identical scalar expression per
//        element (SSE2 lanes do the same IEEE operations; no contraction).
// L's lower triangle holds the running sums until a column is final.
// tests/test_oracle_golden.py pins it bitwise to ldlt() and to the reference.
void ldlt_blocked(int64_t n, const double* A, int64_t lda, double* L, int64_t ldl, double* D) {
  constexpr int64_t NB = 96;
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < n; ++j) {
    for (int64_t i = 0; i <= j; ++i) L[j * ldl + i] = A[j * lda + i];
    for (int64_t i = j + 1; i < n; ++i) L[j * ldl + i] = 0.0;
  }
  std::vector<double> Pt((size_t)(NB * n));  // Pt[kk][i] = L[i][I0 + kk]
  for (int64_t I0 = 0; I0 < n; I0 += NB) {
    const int64_t I1 = std::min(I0 + NB, n);
    for (int64_t i = I0; i < I1; ++i) {  // 1. diagonal block
      const double* Li = L + i * ldl;
      double sum_d = Li[i];
      for (int64_t k = I0; k < i; ++k) sum_d -= Li[k] * Li[k] * D[k];
      D[i] = sum_d == 0.0 ? 1e-8 : sum_d;
      for (int64_t j = i + 1; j < I1; ++j) {
        double* Lj = L + j * ldl;
        double sum = Lj[i];
        for (int64_t k = I0; k < i; ++k) sum -= Lj[k] * Li[k] * D[k];
        Lj[i] = sum / D[i];
      }
      L[i * ldl + i] = 1.0;
    }
    if (I1 >= n) break;
#pragma omp parallel for schedule(static)
    for (int64_t j = I1; j < n; ++j) {  // 2. the panel rows below the block
      double* Lj = L + j * ldl;
      for (int64_t i = I0; i < I1; ++i) {
        const double* Li = L + i * ldl;
        double sum = Lj[i];
        for (int64_t k = I0; k < i; ++k) sum -= Lj[k] * Li[k] * D[k];
        Lj[i] = sum / D[i];
        Pt[(size_t)((i - I0) * n + j)] = Lj[i];
      }
    }
    // 3. trailing triangle, rows in reverse so the long rows start first
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t jj = 0; jj < n - I1; ++jj) {
      const int64_t j = n - 1 - jj;
      double* Sj = L + j * ldl;
      constexpr int64_t IC = 512;  // keep the row chunk in L1 across the k loop
      for (int64_t c0 = I1; c0 <= j; c0 += IC) {
        const int64_t c1 = std::min(c0 + IC, j + 1);
        for (int64_t k = I0; k < I1; ++k) {
          const double ljk = Sj[k], dk = D[k];
          const double* P = Pt.data() + (size_t)((k - I0) * n);
          for (int64_t i = c0; i < c1; ++i) Sj[i] -= ljk * P[i] * dk;
        }
      }
    }
  }
}

void solve_ldlt(int64_t n, const double* L, int64_t ldl, const double* D, double* b) {
  if (n == 0) return;
  for (int64_t i = 0; i < n; ++i) {  // std::inner_product from 0.0
    double s = 0.0;
    for (int64_t j = 0; j < i; ++j) s = s + L[i * ldl + j] * b[j];
    b[i] -= s;
  }
  for (int64_t i = 0; i < n; ++i) b[i] /= D[i];
  for (int64_t i = n - 1; i >= 0; --i) {
    double s = 0.0;
    for (int64_t j = i + 1; j < n; ++j) s += L[j * ldl + i] * b[j];
    b[i] -= s;
  }
}

// get_max_step_ (Optimizer.cpp:270-342): the non-negative Newton variables,
// and -- when neither g nor h is a Newton variable (box-only, or Slacks) --
// explicit bounds on x (l_x, u_x) and s (l_A, u_A); the environment always
// holds both bounds of each, whatever Settings::*_bounds say.
double max_step(const QP& q, const Vec* D) {
  double a = 1.0;
  const int nonneg[8] = {LG, LH, LY, LZ, G, H, Y, Z};
  for (int slot : order(q)) {
    bool nn = false;
    for (int k = 0; k < 8; ++k) nn |= slot == nonneg[k];
    if (!nn) continue;
    for (int64_t j = 0; j < q.size(slot); ++j) {
      const double dij = D[slot][j], vij = q.v[slot][j];
      if (dij < 0.0) a = std::min(a, -vij / dij);
    }
  }
  if (q.size(G) == 0 && q.size(H) == 0) {
    for (int64_t j = 0; j < q.n; ++j) {
      const double dij = D[X][j], vij = q.v[X][j];
      if (dij < 0.0) a = std::min(a, (q.lx[j] - vij) / dij);
      if (dij > 0.0) a = std::min(a, (q.ux[j] - vij) / dij);
    }
    for (int64_t j = 0; j < q.m; ++j) {
      const double dij = D[S][j], vij = q.v[S][j];
      if (dij < 0.0) a = std::min(a, (q.lA[j] - vij) / dij);
      if (dij > 0.0) a = std::min(a, (q.uA[j] - vij) / dij);
    }
  }
  return a;
}

void axpy_all(QP& q, double s, const Vec* D) {
  for (int slot = 0; slot < NSLOT; ++slot)
    for (int64_t j = 0; j < q.size(slot); ++j) q.v[slot][j] = q.v[slot][j] + s * D[slot][j];
}

}  // namespace
static int bk_factor(int64_t n, double* A, int64_t ld, int64_t* ipiv, bool fix_kp);
static void bk_solve(int64_t n, const double* L, int64_t ld, const int64_t* ipiv, double* b);
namespace {

// One Newton iteration (Optimizer.cpp:127-219).  rec = {f, res, mu,
// alpha_aff, mu_aff, sigma, alpha, converged}.
// The factor: ldlt_decomposition for the quasi-definite KKT matrix; for a
// zero diagonal block (EqualityHandling::None, Optimizer.cpp:63-75)
// symmetric_indefinite_factorization + overwriting_solve_bunch_kaufman, with
// the reference's kp = 0 behaviour (fix_kp = false).  L holds F, ipiv the
// pivots, in that case.
// bench.py's cpu_baseline times the reference's own loop order on one core;
// the parity tests take the (bitwise identical) blocked, threaded form
bool g_serial_ldlt = false;

struct Factor {
  Vec L, Dd;
  std::vector<int64_t> ipiv;
};

void search_direction(QP& q, const Residuals& R, const Factor& F, Vec* out) {
  const int64_t N = q.N(), n = q.n, m = q.m;
  Vec b(N);
  augmented_rhs(q, R, b.data());
  if (q.eq_none) bk_solve(N, F.L.data(), N, F.ipiv.data(), b.data());
  else solve_ldlt(N, F.L.data(), N, F.Dd.data(), b.data());
  for (int s = 0; s < NSLOT; ++s) out[s].assign(q.size(s), 0.0);
  std::memcpy(out[X].data(), b.data(), sizeof(double) * n);
  if (q.naive) {
    std::memcpy(out[LG].data(), b.data() + n, sizeof(double) * m);
    std::memcpy(out[LH].data(), b.data() + n + m, sizeof(double) * m);
  } else {
    std::memcpy(out[LA].data(), b.data() + n, sizeof(double) * m);
  }
  std::memcpy(out[LC].data(), b.data() + n + q.mk(), sizeof(double) * q.p);
  back_substitute(q, R, out);
}

int iterate(QP& q, double* rec, double* phase_s) {
  using clk = double;
  (void)sizeof(clk);
  const int64_t N = q.N();
  rec[0] = objective(q);
  rec[1] = residual_norm(q);
  rec[2] = mu_of(q);
  rec[7] = (rec[1] < 1e-8 && rec[2] < 1e-8) ? 1.0 : 0.0;
  if (rec[7] != 0.0) return 1;
  Vec K((size_t)(N * N));
  Factor F;
  const auto t0 = std::chrono::steady_clock::now();
  assemble(q, K.data());
  const auto t1 = std::chrono::steady_clock::now();
  if (q.eq_none) {
    F.ipiv.assign(N, 0);
    bk_factor(N, K.data(), N, F.ipiv.data(), false);
    F.L = std::move(K);
  } else {
    F.L.assign((size_t)(N * N), 0.0);
    F.Dd.assign(N, 0.0);
    if (g_serial_ldlt) ldlt(N, K.data(), N, F.L.data(), N, F.Dd.data());  // the reference's loop order
    else ldlt_blocked(N, K.data(), N, F.L.data(), N, F.Dd.data());    // == ldlt() bit for bit
  }
  const auto t2 = std::chrono::steady_clock::now();
  if (phase_s) {
    phase_s[0] = std::chrono::duration<double>(t1 - t0).count();
    phase_s[1] = std::chrono::duration<double>(t2 - t1).count();
  }
  const double mu = rec[2];
  Residuals R;
  residuals(q, 0.0, R);
  search_direction(q, R, F, q.daff);
  const double a_aff = max_step(q, q.daff);
  Vec saved[NSLOT];
  for (int s = 0; s < NSLOT; ++s) saved[s] = q.v[s];
  axpy_all(q, a_aff, q.daff);
  const double mu_aff = mu_of(q);
  for (int s = 0; s < NSLOT; ++s) q.v[s] = saved[s];
  const double sigma = mu > 0.0 ? std::pow(mu_aff / mu, 3) : 0.0;
  const double mu_new = mu * sigma;
  residuals(q, mu_new, R);
  // Corrector (Optimizer.cpp:183-209): every VARIABLE of a complementarity row
  // replaced by its affine direction, mu by 0, added to the row at mu_new:
  // SlackedSlacks r_g += (dG_aff*dlambda_g_aff) - (0*e); Slacks r_lambda_y +=
  // ((dX_aff - L_x)*dlambda_y_aff) - (0*e) -- the bound constant leaks in
  // (the reference's Slacks defect, reproduced)
  {
    const Vec* dv = q.daff;
    for (int64_t i = 0; i < q.size(G); ++i) R.r[G][i] = R.r[G][i] + (dv[G][i] * dv[LG][i] + (-(0.0 * 1.0)));
    for (int64_t i = 0; i < q.size(H); ++i) R.r[H][i] = R.r[H][i] + (dv[H][i] * dv[LH][i] + (-(0.0 * 1.0)));
    for (int64_t i = 0; i < q.size(Y); ++i) R.r[Y][i] = R.r[Y][i] + (dv[Y][i] * dv[LY][i] + (-(0.0 * 1.0)));
    for (int64_t i = 0; i < q.size(Z); ++i) R.r[Z][i] = R.r[Z][i] + (dv[Z][i] * dv[LZ][i] + (-(0.0 * 1.0)));
    if (q.slacks) {
      for (int64_t i = 0; i < q.size(LG); ++i)
        R.r[LG][i] = R.r[LG][i] + ((dv[S][i] + (-q.lA[i])) * dv[LG][i] + (-(0.0 * 1.0)));
      for (int64_t i = 0; i < q.size(LH); ++i)
        R.r[LH][i] = R.r[LH][i] + ((q.uA[i] + (-dv[S][i])) * dv[LH][i] + (-(0.0 * 1.0)));
      for (int64_t i = 0; i < q.size(LY); ++i)
        R.r[LY][i] = R.r[LY][i] + ((dv[X][i] + (-q.lx[i])) * dv[LY][i] + (-(0.0 * 1.0)));
      for (int64_t i = 0; i < q.size(LZ); ++i)
        R.r[LZ][i] = R.r[LZ][i] + ((q.ux[i] + (-dv[X][i])) * dv[LZ][i] + (-(0.0 * 1.0)));
    }
  }
  search_direction(q, R, F, q.dir);
  const double alpha = max_step(q, q.dir);
  axpy_all(q, 0.995 * alpha, q.dir);
  if (phase_s) phase_s[2] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t2).count();
  rec[3] = a_aff;
  rec[4] = mu_aff;
  rec[5] = sigma;
  rec[6] = alpha;
  q.mu = mu_new;
  return 0;
}

}  // namespace

// ===========================================================================
// Bunch-Kaufman (LinearSolvers.cpp:76-207 factor, :209-318 solve), restated:
// LAPACK dsytf2-'L' style diagonal pivoting with alpha = (1 + sqrt 17) / 8,
// in place on a full row-major matrix (only the lower triangle is touched).
// ipiv: >= 0 a 1x1 pivot with that interchange, < 0 (-kp, twice) a 2x2.
// fix_kp = false reproduces the reference exactly, including its defect of
// leaving kp = 0 for a second all-zero column (LinearSolvers.cpp:111-116);
// fix_kp = true records kp = k there (what LAPACK does).
namespace {
struct ArgMax {
  int64_t idx;
  double val;
};
// largest |.| over i in [b, e) of column c (col) or row r (!col); ties keep
// the first index (strictly-greater scan from b)
ArgMax absmax(const double* A, int64_t ld, int64_t b, int64_t e, int64_t fixed, bool col) {
  ArgMax m{0, 0.0};
  for (int64_t i = b; i < e; ++i) {
    const double v = std::fabs(col ? A[i * ld + fixed] : A[fixed * ld + i]);
    if (v > m.val) m = {i, v};
  }
  return m;
}
}  // namespace

static std::vector<double> a_col(const double* A, int64_t ld, int64_t k, int64_t n) {
  std::vector<double> c(n, 0.0);
  for (int64_t i = k; i < n; ++i) c[i] = A[i * ld + k];
  return c;
}

static int bk_factor(int64_t n, double* A, int64_t ld, int64_t* ipiv, bool fix_kp) {
  const double alpha = (1.0 + std::sqrt(17.0)) / 8.0;
  auto a = [&](int64_t i, int64_t j) -> double& { return A[i * ld + j]; };
  int info = 0;
  for (int64_t k = 0; k < n;) {
    int step = 1;
    int64_t kp = 0;
    const double akk = std::fabs(a(k, k));
    const ArgMax cm = absmax(A, ld, k + 1, n, k, true);
    if (akk == 0.0 && cm.val == 0.0) {
      if (info == 0) {
        info = (int)k;
        kp = k;
      } else if (fix_kp) {
        kp = k;
      }
    } else {
      if (akk >= alpha * cm.val) {
        kp = k;
      } else {
        const double rmax = std::max(absmax(A, ld, k, cm.idx, cm.idx, false).val,
                                     absmax(A, ld, cm.idx + 1, n, cm.idx, true).val);
        if (akk * rmax >= alpha * cm.val * cm.val) kp = k;
        else if (std::fabs(a(cm.idx, cm.idx)) >= alpha * rmax) kp = cm.idx;
        else {
          kp = cm.idx;
          step = 2;
        }
      }
      const int64_t kk = k + step - 1;
      if (kp != kk) {  // symmetric interchange of kk and kp in A(k:n, k:n), lower part
        for (int64_t i = kp + 1; i < n; ++i) std::swap(a(i, kp), a(i, kk));
        for (int64_t j = kk + 1; j < kp; ++j) std::swap(a(kp, j), a(j, kk));
        std::swap(a(kp, kp), a(kk, kk));
        if (step == 2) std::swap(a(kk, k), a(kp, k));
      }
      // The updates below are the reference's loops (LinearSolvers.cpp:155-192)
      // with the (j, i) loops exchanged: every element gets the same single
      // expression from the same unscaled pivot-column values (staged first,
      // since the reference scales a(j, k) only after its column j), so the
      // result is bitwise the serial loop's; rows run in parallel.
      const int64_t j0 = k + step;
      std::vector<double> c0(a_col(A, ld, k, n)), c1(step == 2 ? a_col(A, ld, k + 1, n) : std::vector<double>());
      if (step == 1) {  // rank-1: A -= W (1/d) W^T, column k -> L(k)
        const double r = 1.0 / a(k, k);
        std::vector<double> f(n);
        for (int64_t j = j0; j < n; ++j) f[j] = r * c0[j];
#pragma omp parallel for schedule(dynamic, 32) if (n - k > 512)
        for (int64_t i = j0; i < n; ++i) {
          double* Ai = A + i * ld;
          const double ci = c0[i];
          for (int64_t j = j0; j <= i; ++j) Ai[j] -= f[j] * ci;
          Ai[k] *= r;
        }
      } else if (k < n - 1) {  // rank-2 with the inverse of the 2x2 block
        double d21 = a(k + 1, k);
        const double d11 = a(k + 1, k + 1) / d21;
        const double d22 = a(k, k) / d21;
        const double t = 1.0 / (d11 * d22 - 1.0);
        d21 = t / d21;
        std::vector<double> wk(n), wk1(n);
        for (int64_t j = j0; j < n; ++j) {
          wk[j] = d21 * (d11 * c0[j] - c1[j]);
          wk1[j] = d21 * (d22 * c1[j] - c0[j]);
        }
#pragma omp parallel for schedule(dynamic, 32) if (n - k > 512)
        for (int64_t i = j0; i < n; ++i) {
          double* Ai = A + i * ld;
          const double ui = c0[i], vi = c1[i];
          for (int64_t j = j0; j <= i; ++j) Ai[j] -= (ui * wk[j] + vi * wk1[j]);
          Ai[k] = wk[i];
          Ai[k + 1] = wk1[i];
        }
      }
    }
    if (step == 1) ipiv[k] = kp;
    else ipiv[k] = ipiv[k + 1] = -kp;
    k += step;
  }
  return info;
}

static void bk_solve(int64_t n, const double* L, int64_t ld, const int64_t* ipiv, double* b) {
  if (n == 0) return;
  auto l = [&](int64_t i, int64_t j) { return L[i * ld + j]; };
  auto axpy_col = [&](int64_t from, int64_t j) {  // b[from:] -= L[from:, j] b[j]
    const double mlt = -b[j];
    for (int64_t i = from; i < n; ++i) b[i] += l(i, j) * mlt;
  };
  for (int64_t k = 0; k < n;) {  // L D y = P b
    if (ipiv[k] >= 0) {
      const int64_t kp = ipiv[k];
      if (kp != k) std::swap(b[k], b[kp]);
      axpy_col(k + 1, k);
      b[k] /= l(k, k);
      k += 1;
    } else {
      const int64_t kp = -ipiv[k];
      if (kp != k + 1) std::swap(b[k + 1], b[kp]);
      if (k < n - 1) {
        axpy_col(k + 2, k);
        axpy_col(k + 2, k + 1);
      }
      const double d21 = l(k + 1, k);
      const double d11 = l(k, k) / d21;
      const double d22 = l(k + 1, k + 1) / d21;
      const double den = d11 * d22 - 1.0;
      const double b1 = b[k] / d21, b2 = b[k + 1] / d21;
      b[k] = (d22 * b1 - b2) / den;
      b[k + 1] = (d11 * b2 - b1) / den;
      k += 2;
    }
  }
  auto dot_col = [&](int64_t from, int64_t j) {  // b[j] -= L[from:, j] . b[from:]
    double s = 0.0;
    for (int64_t i = from; i < n; ++i) s += l(i, j) * b[i];
    b[j] -= s;
  };
  for (int64_t k = n - 1; k >= 0;) {  // L^T x = y, then undo the interchanges
    if (ipiv[k] >= 0) {
      if (k < n - 1) dot_col(k + 1, k);
      const int64_t kp = ipiv[k];
      if (kp != k) std::swap(b[k], b[kp]);
      k -= 1;
    } else {
      if (k < n - 1) {
        dot_col(k + 1, k);
        dot_col(k + 1, k - 1);
      }
      const int64_t kp = -ipiv[k];
      if (kp != k) std::swap(b[k], b[kp]);
      k -= 2;
    }
  }
}

// ===========================================================================
// C ABI for ctypes (tests, smoke, bench cpu_baseline)
extern "C" {

int ipmzo_bk_factor(int64_t n, double* A, int64_t ld, int64_t* ipiv, int fix_kp) {
  return bk_factor(n, A, ld, ipiv, fix_kp != 0);
}
void ipmzo_bk_solve(int64_t n, const double* F, int64_t ld, const int64_t* ipiv, double* b) {
  bk_solve(n, F, ld, ipiv, b);
}

void ipmzo_gen_qp(int64_t n, int64_t m, int64_t p, uint64_t seed, double* Q, double* c, double* A, double* lA,
                  double* uA, double* C, double* d, double* lx, double* ux) {
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t j = 0; j < i; ++j) {
      const double v = (2.0 * u01(seed, TAG_Q, i, j) - 1.0) / (double)n;
      Q[i * n + j] = v;
      Q[j * n + i] = v;
    }
    Q[i * n + i] = 1.0 + u01(seed, TAG_Q, i, i);
    c[i] = 2.0 * u01(seed, TAG_C, i, 0) - 1.0;
    lx[i] = -1.0;
    ux[i] = 1.0;
  }
  const double sn = std::sqrt((double)n);
  for (int64_t i = 0; i < m; ++i) {
    for (int64_t j = 0; j < n; ++j) A[i * n + j] = (2.0 * u01(seed, TAG_A, i, j) - 1.0) / sn;
    lA[i] = -1.0;
    uA[i] = 1.0;
  }
  for (int64_t i = 0; i < p; ++i) {
    for (int64_t j = 0; j < n; ++j) C[i * n + j] = (2.0 * u01(seed, TAG_C_EQ, i, j) - 1.0) / sn;
    d[i] = (2.0 * u01(seed, TAG_D, i, 0) - 1.0) * 0.1;
  }
}

double ipmzo_u01(uint64_t seed, uint64_t tag, uint64_t i, uint64_t j) { return u01(seed, tag, i, j); }

void ipmzo_ldlt(int64_t n, const double* A, int64_t lda, double* L, int64_t ldl, double* D) {
  ldlt(n, A, lda, L, ldl, D);
}
void ipmzo_set_serial_ldlt(int serial) { g_serial_ldlt = serial != 0; }
void ipmzo_ldlt_blocked(int64_t n, const double* A, int64_t lda, double* L, int64_t ldl, double* D) {
  ldlt_blocked(n, A, lda, L, ldl, D);
}
void ipmzo_solve_ldlt(int64_t n, const double* L, int64_t ldl, const double* D, double* b) {
  solve_ldlt(n, L, ldl, D, b);
}

void* ipmzo_create(int64_t n, int64_t m, int64_t p, const double* Q, const double* c, const double* A,
                   const double* lA, const double* uA, const double* C, const double* d, const double* lx,
                   const double* ux) {
  auto* q = new QP();
  q->n = n;
  q->m = m;
  q->p = p;
  q->delta = 1e-4;
  q->mu = 1.0;
  q->Q.assign(Q, Q + n * n);
  q->c.assign(c, c + n);
  q->A.assign(A, A + m * n);
  q->lA.assign(lA, lA + m);
  q->uA.assign(uA, uA + m);
  q->C.assign(C, C + p * n);
  q->d.assign(d, d + p);
  q->lx.assign(lx, lx + n);
  q->ux.assign(ux, ux + n);
  // build_environment initial iterate (EnvironmentBuilder.cpp:34-73)
  for (int s = 0; s < NSLOT; ++s) {
    q->v[s].assign(q->size(s), 1.0);
    q->daff[s].assign(q->size(s), 0.0);
    q->dir[s].assign(q->size(s), 0.0);
  }
  for (int64_t i = 0; i < n; ++i) q->v[X][i] = 0.5 * (lx[i] + ux[i]);
  for (int64_t i = 0; i < m; ++i) q->v[S][i] = 0.5 * (lA[i] + uA[i]);
  return q;
}

void ipmzo_destroy(void* h) { delete static_cast<QP*>(h); }

// EqualityHandling::None (call right after ipmzo_create): drops p, zero
// (lambda_C, lambda_C) block, Bunch-Kaufman factor.
void ipmzo_set_equality_penalty(void* h) {
  QP& q = *static_cast<QP*>(h);
  q.eq_pen = true;
  q.v[P].clear();
  q.daff[P].clear();
  q.dir[P].clear();
}
void ipmzo_set_equality_none(void* h) {
  QP& q = *static_cast<QP*>(h);
  q.eq_none = true;
  q.v[P].clear();
  q.daff[P].clear();
  q.dir[P].clear();
}

// Settings (call right after ipmzo_create): inequality handling (0
// SlackedSlacks, 1 Slacks) and the bounds (IPMZ_BOUNDS_*: 0 None, 1 Lower,
// 2 Upper, 3 Both) of the inequalities and of the variables.  Resizes the
// slots and restores build_environment's initial iterate.
// handling: 0 SlackedSlacks, 1 Slacks, 2 NaiveSlacks
int ipmzo_set_formulation(void* h, int handling, int ineq_bounds, int var_bounds) {
  QP& q = *static_cast<QP*>(h);
  if (q.m > 0 && ineq_bounds == 0) return -1;  // the reference then drops A entirely: not modelled
  q.slacks = handling == 1;
  q.naive = handling == 2;
  if (q.naive && q.m > 0 && ineq_bounds != 3) return -1;  // NaiveSlacks: both inequality bounds
  q.alo = (ineq_bounds & 1) != 0;
  q.aup = (ineq_bounds & 2) != 0;
  q.vlo = (var_bounds & 1) != 0;
  q.vup = (var_bounds & 2) != 0;
  if (q.slacks && (!q.alo || !q.aup || !q.vlo || !q.vup)) return -1;  // Slacks: Bounds::Both only (pinned)
  for (int s = 0; s < NSLOT; ++s) {
    q.v[s].assign(q.size(s), 1.0);
    q.daff[s].assign(q.size(s), 0.0);
    q.dir[s].assign(q.size(s), 0.0);
  }
  for (int64_t i = 0; i < q.n; ++i) q.v[X][i] = 0.5 * (q.lx[i] + q.ux[i]);
  for (int64_t i = 0; i < q.m && !q.naive; ++i) q.v[S][i] = 0.5 * (q.lA[i] + q.uA[i]);
  return 0;
}

int64_t ipmzo_kkt_dim(void* h) { return static_cast<QP*>(h)->N(); }

int ipmzo_iterate(void* h, double* rec) { return iterate(*static_cast<QP*>(h), rec, nullptr); }
// phase_s = {assemble, ldlt, rest-of-step (rhs, 2 solves, back-substitution,
// ratio tests, update)} in seconds; the head (objective, residual norm, mu)
// is included in neither.
int ipmzo_iterate_timed(void* h, double* rec, double* phase_s) { return iterate(*static_cast<QP*>(h), rec, phase_s); }

// Concatenated vectors in the reference's Newton-variable order.
int64_t ipmzo_state_len(void* h) {
  const QP& q = *static_cast<QP*>(h);
  int64_t t = 0;
  for (int s : order(q)) t += q.size(s);
  return t;
}
static void pack(const QP& q, const Vec* src, double* out) {
  for (int s : order(q)) {
    std::memcpy(out, src[s].data(), sizeof(double) * q.size(s));
    out += q.size(s);
  }
}
void ipmzo_get_vars(void* h, double* out) { const QP& q = *static_cast<QP*>(h); pack(q, q.v, out); }
void ipmzo_get_daff(void* h, double* out) { const QP& q = *static_cast<QP*>(h); pack(q, q.daff, out); }
void ipmzo_get_dir(void* h, double* out) { const QP& q = *static_cast<QP*>(h); pack(q, q.dir, out); }
void ipmzo_set_vars(void* h, const double* in) {
  QP& q = *static_cast<QP*>(h);
  for (int s : order(q)) {
    std::memcpy(q.v[s].data(), in, sizeof(double) * q.size(s));
    in += q.size(s);
  }
}
void ipmzo_assemble(void* h, double* K) { assemble(*static_cast<QP*>(h), K); }
void ipmzo_rhs(void* h, double mu, double* b) {
  QP& q = *static_cast<QP*>(h);
  Residuals R;
  residuals(q, mu, R);
  augmented_rhs(q, R, b);
}
double ipmzo_residual_norm(void* h) { return residual_norm(*static_cast<QP*>(h)); }
double ipmzo_mu(void* h) { return mu_of(*static_cast<QP*>(h)); }
double ipmzo_objective(void* h) { return objective(*static_cast<QP*>(h)); }

}  // extern "C"
