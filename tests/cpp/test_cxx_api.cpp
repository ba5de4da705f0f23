// C++ API test (reference-style, gtest-free): the mirrored
// NumericalOptimization interface over libipmz, on the GPU.  Built and run by
// tests/test_gpu_cxx.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "ipmz/NumericalOptimization.hpp"

using namespace ipmz::NumericalOptimization;

#define EXPECT(cond)                                                  \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

int main() {
  // LDL^T of a small quasi-definite matrix, then solve (LinearSolvers.cpp:14-74)
  Matrix K = {{4.0, 1.0, 2.0}, {1.0, 3.0, 0.5}, {2.0, 0.5, -1.0}};
  auto [L, D] = LinearSolvers::ldlt_decomposition(K);
  EXPECT(L[0][0] == 1.0 && L[1][1] == 1.0 && L[0][1] == 0.0);
  EXPECT(std::fabs(D[0] - 4.0) < 1e-15);
  EXPECT(std::fabs(L[1][0] - 0.25) < 1e-15);
  Vector b = {1.0, 2.0, 3.0};
  LinearSolvers::overwriting_solve_ldlt(L, D, b);
  for (int i = 0; i < 3; ++i) {
    double r = -(i == 0 ? 1.0 : i == 1 ? 2.0 : 3.0);
    for (int j = 0; j < 3; ++j) r += K[i][j] * b[j];
    EXPECT(std::fabs(r) < 1e-13);
  }
  // a non-square matrix throws AssertionError (a std::logic_error)
  bool threw = false;
  try {
    LinearSolvers::ldlt_decomposition(Matrix{{1.0, 2.0}});
  } catch (const std::logic_error&) {
    threw = true;
  }
  EXPECT(threw);
  // empty b is a no-op
  Vector e;
  LinearSolvers::overwriting_solve_ldlt(Matrix{}, Vector{}, e);

  // The IpmZoo -n style QP with SlackedSlacks (IpmZoo.cpp:359-370 data; the
  // shipped example uses the stagnating Slacks formulation)
  Data d;
  d.Q = {{1.0, 0.0}, {0.0, 0.5}};
  d.c = {-10.0, 2.0};
  d.A_ineq = {{1.0, 1.0}};
  d.l_A_ineq = {1.0};
  d.u_A_ineq = {1.2};
  d.l_x = {0.0, 0.0};
  d.u_x = {10.0, 10.0};
  Optimizer opt(d);
  auto trace = opt.solve();
  EXPECT(!trace.empty() && trace.size() < 100);
  auto x = opt.x();
  // optimum: x1 + x2 <= 1.2 active, x2 at 0 -> x = (1.2, 0)
  EXPECT(std::fabs(x[0] - 1.2) < 1e-6 && std::fabs(x[1]) < 1e-6);

  // the same optimum with only the active sides of the bounds (Settings,
  // SymbolicOptimization.h:58-64): x1 + x2 <= 1.2 and x >= 0
  Settings st;
  st.inequalities = Bounds::Upper;
  st.variable_bounds = Bounds::Lower;
  Optimizer one_sided(d, st);
  auto trace1 = one_sided.solve();
  auto x1 = one_sided.x();
  EXPECT(!trace1.empty() && trace1.size() < 100);
  EXPECT(std::fabs(x1[0] - 1.2) < 1e-6 && std::fabs(x1[1]) < 1e-6);
  EXPECT(one_sided.variables().size() == 2 + 2 * 2 + 4 * 1);  // x, lambda_y, y; lambda_A, s, lambda_h, h
  // Slacks is built on both bounds: one-sided settings are rejected
  st.inequality_handling = InequalityHandling::Slacks;
  threw = false;
  try {
    Optimizer o3(d, st);
  } catch (const ipmz::AssertionError&) {
    threw = true;
  }
  EXPECT(threw);

  // build_environment validation: l_x < u_x (EnvironmentBuilder.cpp:12-14)
  Data bad = d;
  bad.u_x = {0.0, 10.0};
  threw = false;
  try {
    Optimizer o2(bad);
  } catch (const ipmz::AssertionError&) {
    threw = true;
  }
  EXPECT(threw);
  std::printf("cxx api ok: %zu iterations, x = (%.9f, %.9f)\n", trace.size(), x[0], x[1]);
  return 0;
}
