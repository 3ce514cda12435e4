// ipm_host.cpp -- DEVELOPMENT TOOL ONLY: the lane routine of ipm.hip
// (ipm_lane.hpp) compiled for the host CPU, so the interior-point algorithm
// can be stepped through and compared with the oracle without a GPU.  It is
// not part of libmpcqp.so and nothing in the package, tests or bench loads it.
//   g++ -O2 -shared -fPIC -I include tools/ipm_host.cpp -o /tmp/libipm_host.so
#define MPCQP_HD
#include <cstdlib>
#include <vector>

#include "../include/mpcqp.h"
#include "../model_predictive_control_amd/csrc/ipm_lane.hpp"

using namespace mpcqp;

extern "C" int ipm_host_solve(int batch, int nx, int nu, int N, int tv, const double* A,
                              long sA, const double* B, long sB, const double* c, long sC,
                              const double* Q, const double* R, const double* Qf,
                              const double* x0, const double* xlo, const double* xhi,
                              const double* lb, const double* ub, double* z, double* y, double* X,
                              int* status, int max_iter, double tol, const double* H2,
                              const double* q2, double* pi) {
  ipm::Args<double> a{};
  a.batch = batch; a.nx = nx; a.nu = nu; a.N = N; a.tv = tv;
  a.max_iter = max_iter; a.tol = tol; a.tol_mu = 1e-2 * tol; a.tol_polish = 1e-6; a.mu_polish = getenv("MUP") ? atof(getenv("MUP")) : 1e-6;
  a.strict = getenv("STRICT") ? atoi(getenv("STRICT")) : 0;
  a.A = A; a.sA = sA; a.B = B; a.sB = sB; a.c = c; a.sC = sC;
  a.Q = Q; a.R = R; a.Qf = Qf; a.x0 = x0; a.sX0 = nx;
  a.xlo = xlo; a.xhi = xhi; a.sXb = 0; a.lb = lb; a.ub = ub;
  a.z = z; a.y = y; a.X = X; a.status = status;
  a.H2 = H2; a.sH2 = 0; a.q2 = q2; a.sq2 = 0; a.pi = pi;
  const bool small = nx <= 2 && nu <= 1;
  const int F = small ? ipm::Layout<2, 1>::F : ipm::Layout<4, 2>::F;
  std::vector<double> ws((size_t)N * F * batch);
  a.ws = ws.data();
  for (int b = 0; b < batch; ++b) {
    if (small) ipm::solve_lane<double, 2, 1, 1>(a, b, ws.data() + (size_t)b * N * F);
    else ipm::solve_lane<double, 4, 2, 1>(a, b, ws.data() + (size_t)b * N * F);
  }
  return 0;
}
