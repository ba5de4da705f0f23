// C++ mirror of the reference's NumericalOptimization interface for the hot
// path, over the C ABI of libipmz (include/ipmz.h).  Header-only.
//
//   LinearSolvers::ldlt_decomposition      include/NumericalOptimization/LinearSolvers.h:11
//   LinearSolvers::overwriting_solve_ldlt  LinearSolvers.h:16-17
//   Data, build_environment                EnvironmentBuilder.h:7-20
//   Optimizer(...).solve()                 Optimizer.h:15-20
//
// Same names, argument meaning and error behaviour: value-returning factor
// (fresh L and D), in-place solve, and failures thrown as AssertionError,
// a std::logic_error (Utils::AssertionError, Assert.h:7-12).  Formulation:
// Settings below (default SlackedSlacks, Bounds::Both, Regularization when
// equality rows are present); Settings the numeric path cannot run (SURVEY.md
// §0.3) are rejected with AssertionError.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "ipmz.h"

namespace ipmz {

struct AssertionError : std::logic_error {
  using std::logic_error::logic_error;
};

inline int check(int rc, const char* what) {
  if (rc < 0) throw AssertionError(std::string(what) + ": " + ipmz_last_error());
  return rc;
}

// One device + stream.  Not thread-safe; one per thread / GPU.
class Context {
 public:
  explicit Context(int device = 0) { check(ipmz_ctx_create(&h_, device), "ipmz_ctx_create"); }
  ~Context() { ipmz_ctx_destroy(h_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  ipmz_ctx* get() const { return h_; }
  static Context& instance() {
    static Context c(0);
    return c;
  }

 private:
  ipmz_ctx* h_ = nullptr;
};

namespace NumericalOptimization {
using Matrix = std::vector<std::vector<double>>;
using Vector = std::vector<double>;

namespace LinearSolvers {

// LDL^T of a symmetric matrix (lower triangle read); returns L (full N x N,
// unit diagonal, zeros above) and D.  Vanderbei's zero-pivot rule applies.
inline std::pair<Matrix, Vector> ldlt_decomposition(const Matrix& A, Context& ctx = Context::instance()) {
  const size_t n = A.size();
  for (const auto& row : A)
    if (row.size() != n) throw AssertionError("ldlt_decomposition: matrix is not square");  // LinearSolvers.cpp:16-17
  std::vector<double> flat(n * n), L(n * n), D(n);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) flat[i * n + j] = A[i][j];
  check(ipmz_ldlt_decomposition(ctx.get(), (int)n, flat.data(), L.data(), D.data()), "ipmz_ldlt_decomposition");
  Matrix Lm(n, Vector(n));
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) Lm[i][j] = L[i * n + j];
  return {std::move(Lm), std::move(D)};
}

// Solves (L D L^T) x = b, overwriting b.  Empty b is a no-op.
inline void overwriting_solve_ldlt(const Matrix& L, const Vector& D, Vector& b, Context& ctx = Context::instance()) {
  if (b.empty()) return;  // LinearSolvers.cpp:46-48
  const size_t n = b.size();
  if (D.size() != n || L.size() != n) throw AssertionError("overwriting_solve_ldlt: size mismatch");
  std::vector<double> flat(n * n);
  for (size_t i = 0; i < n; ++i) {
    if (L[i].size() != n) throw AssertionError("overwriting_solve_ldlt: L is not square");
    for (size_t j = 0; j < n; ++j) flat[i * n + j] = L[i][j];
  }
  check(ipmz_overwriting_solve_ldlt(ctx.get(), (int)n, flat.data(), D.data(), b.data()), "ipmz_overwriting_solve_ldlt");
}

}  // namespace LinearSolvers

// EnvironmentBuilder.h:7-17
struct Data {
  Matrix Q;
  Vector c;
  Matrix A_ineq;
  Vector l_A_ineq;
  Vector u_A_ineq;
  Matrix A_eq;
  Vector b_eq;
  Vector l_x;
  Vector u_x;
};

struct IterationRecord {
  double f, res, mu, alpha_aff, mu_aff, sigma, alpha;
};

// Settings::EqualityHandling (SymbolicOptimization.h:41-49), the three the
// numeric path supports: Regularization (quasi-definite, LDL^T), None (the
// reference's default: zero diagonal block, Optimizer::solve's indefinite
// branch, Optimizer.cpp:63-75, on the Bunch-Kaufman factor) and
// PenaltyFunction (-mu I block, LDL^T)
enum class EqualityHandling {
  Regularization = IPMZ_EQ_REGULARIZATION,
  None = IPMZ_EQ_NONE,
  PenaltyFunction = IPMZ_EQ_PENALTY,
  PenaltyFunctionWithExtraDual = IPMZ_EQ_PENALTY_EXTRA_DUAL,  // the same Newton system (SymbolicOptimization.cpp:364-366)
  SlackedSlacks = IPMZ_EQ_SLACKED_SLACKS,
  NaiveSlacks = IPMZ_EQ_NAIVE_SLACKS  // with InequalityHandling::NaiveSlacks
};

// Settings::Bounds and Settings::InequalityHandling (SymbolicOptimization.h:
// 28-39): SlackedSlacks, Slacks (Both bounds only) and NaiveSlacks (both
// inequality bounds).
enum class Bounds { None = IPMZ_BOUNDS_NONE, Lower = IPMZ_BOUNDS_LOWER, Upper = IPMZ_BOUNDS_UPPER, Both = IPMZ_BOUNDS_BOTH };
enum class InequalityHandling {
  Slacks = IPMZ_INEQ_SLACKS,
  SlackedSlacks = IPMZ_INEQ_SLACKED_SLACKS,
  NaiveSlacks = IPMZ_INEQ_NAIVE_SLACKS
};

// The subset of Settings (SymbolicOptimization.h:58-64) that selects the
// Newton system; defaults are this library's (Regularization when equality
// rows exist), not the reference's EqualityHandling::None.
struct Settings {
  Bounds inequalities = Bounds::Both;
  Bounds variable_bounds = Bounds::Both;
  EqualityHandling equality_handling = EqualityHandling::Regularization;
  InequalityHandling inequality_handling = InequalityHandling::SlackedSlacks;
};

// build_environment + Optimizer: the iterate lives in device memory; solve()
// runs Optimizer.cpp:124-219 (tolerance 1e-8, at most 100 iterations).
class Optimizer {
 public:
  explicit Optimizer(const Data& d, Context& ctx = Context::instance(),
                     EqualityHandling eq = EqualityHandling::Regularization)
      : Optimizer(d, Settings{Bounds::Both, Bounds::Both, eq, InequalityHandling::SlackedSlacks}, ctx) {}
  Optimizer(const Data& d, const Settings& st, Context& ctx = Context::instance()) {
    const int n = (int)d.Q.size(), m = (int)d.A_ineq.size(), p = (int)d.A_eq.size();
    n_ = n;
    ipmz_qp_config cfg{n,
                       m,
                       p,
                       1e-4,
                       static_cast<int>(st.equality_handling),
                       static_cast<int>(st.inequality_handling),
                       static_cast<int>(st.inequalities),
                       static_cast<int>(st.variable_bounds)};
    check(ipmz_qp_create(ctx.get(), &cfg, &h_), "ipmz_qp_create");
    auto flat = [](const Matrix& M, size_t cols) {
      std::vector<double> f;
      f.reserve(M.size() * cols);
      for (const auto& r : M) {
        if (r.size() != cols) throw AssertionError("Data: ragged matrix");
        f.insert(f.end(), r.begin(), r.end());
      }
      return f;
    };
    if (d.c.size() != (size_t)n || d.l_x.size() != (size_t)n || d.u_x.size() != (size_t)n ||
        d.l_A_ineq.size() != (size_t)m || d.u_A_ineq.size() != (size_t)m || d.b_eq.size() != (size_t)p)
      throw AssertionError("Data: inconsistent sizes");
    const auto Q = flat(d.Q, n), A = flat(d.A_ineq, n), C = flat(d.A_eq, n);
    try {
      check(ipmz_qp_load_host(h_, Q.data(), d.c.data(), m ? A.data() : nullptr, m ? d.l_A_ineq.data() : nullptr,
                              m ? d.u_A_ineq.data() : nullptr, p ? C.data() : nullptr, p ? d.b_eq.data() : nullptr,
                              d.l_x.data(), d.u_x.data()),
            "build_environment");
    } catch (...) {
      ipmz_qp_destroy(h_);
      throw;
    }
  }
  ~Optimizer() { ipmz_qp_destroy(h_); }
  Optimizer(const Optimizer&) = delete;
  Optimizer& operator=(const Optimizer&) = delete;

  // Optimizer::solve (Optimizer.cpp:63-73).  Returns the per-iteration trace.
  std::vector<IterationRecord> solve(int max_iter = 100) {
    std::vector<double> tr(8 * (size_t)(max_iter + 1));
    int it = 0;
    check(ipmz_qp_solve(h_, max_iter, tr.data(), &it), "ipmz_qp_solve");
    std::vector<IterationRecord> out;
    for (int i = 0; i <= it && i < max_iter; ++i)
      out.push_back({tr[8 * i], tr[8 * i + 1], tr[8 * i + 2], tr[8 * i + 3], tr[8 * i + 4], tr[8 * i + 5], tr[8 * i + 6]});
    return out;
  }
  void step() { check(ipmz_qp_step(h_, 0), "ipmz_qp_step"); }
  // Newton-order concatenation of the iterate (x first).
  Vector variables() const {
    Vector v((size_t)ipmz_qp_state_len(h_));
    check(ipmz_qp_get_state(h_, IPMZ_STATE_VARS, v.data()), "ipmz_qp_get_state");
    return v;
  }
  Vector x() const {
    Vector v = variables();
    v.resize((size_t)n_);
    return v;
  }
  int n() const { return n_; }

 private:
  ipmz_qp* h_ = nullptr;
  int n_ = 0;
};

}  // namespace NumericalOptimization
}  // namespace ipmz
