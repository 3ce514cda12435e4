// Per-stage cycle counts of the wave interior point's recursions
// (ipm_wave.hpp) on one wave, stage data random but well-posed (SPD weights):
// clock64 (core clock) around riccati_mfma, forward_mfma, rhs_mfma at N = 30.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define MPCQP_HD __host__ __device__
#include "../../model_predictive_control_amd/csrc/common.hpp"
#include "../../model_predictive_control_amd/csrc/ipm_lane.hpp"
#include "../../model_predictive_control_amd/csrc/ipm_quad.hpp"
#include "../../model_predictive_control_amd/csrc/ipm_wave.hpp"
using namespace mpcqp;
using L = ipmq::L;
constexpr int N = 30;
// s_memtime (core clock): each mark also waits for the LDS operations in
// flight (the counter returns through lgkmcnt), so load latency shows in the
// segment that follows the loads
__device__ __forceinline__ unsigned cyc() { return (unsigned)__builtin_amdgcn_s_memtime(); }
using ipmq::NX; using ipmq::NU; using ipmq::pk; using ipmq::inv2;
template <int FGX, int FGU, int FSX, int FSU>
__device__ __attribute__((always_inline)) bool ric_t(double* W, int N, double dreg, unsigned* seg) {
  using namespace mpcqp::ipmw;
  unsigned tprev = cyc();
  const int lane = (int)threadIdx.x;
  const int r = lane >> 4, c = lane & 3;
  const bool store = ((lane >> 2) & 3) == 0;
  const bool isB = c < 2, isE = c == 2, isD = r == c, rowU = r < 2;
  // lane-constant offsets of the lane's element in a stage's fields
  const int oA = L::DA + r * NX + c;
  const int oB = L::DB + r * NU + (c & 1);
  const int oE = L::E + r;
  const int oWXX = L::WXX + pk(r, c);
  const int oSX = FSX + r, oGX = FGX + r;
  const int oWXU = L::WXU + c * NU + (r & 1);
  const int oPP = L::PP + pk(r, c), oKM = L::KM + (r & 1) * NX + c;
  // the stage's operands, loaded one stage ahead (the LDS round trip then
  // overlaps the previous stage's products instead of opening each stage)
  struct Ops {
    double a, bq, e, wxx, sx, gx, wxu, wuu0, wuu1, wuu2, su0, su1, gu0, gu1;
  };
  auto load = [&](int k) {
    const double* S = W + k * L::F;
    Ops o;
    o.a = S[oA]; o.bq = S[oB]; o.e = S[oE]; o.wxx = S[oWXX];
    o.sx = S[oSX]; o.gx = S[oGX]; o.wxu = S[oWXU];
    o.wuu0 = S[L::WUU]; o.wuu1 = S[L::WUU + 1]; o.wuu2 = S[L::WUU + 2];
    o.su0 = S[FSU]; o.su1 = S[FSU + 1]; o.gu0 = S[FGU]; o.gu1 = S[FGU + 1];
    return o;
  };
  double Ph = 0.0, phc = 0.0;
  bool ok = true;
  Ops nx = load(N - 1);
  for (int k = N - 1; k >= 0; --k) {
    double* S = W + k * L::F;
    const Ops o = nx;
    // P = Q' + H2xx + Ph + Sigma_x (+ shift), p = g_x + ph (column 2)
    const double P = o.wxx + Ph + (isD ? o.sx + dreg : 0.0);
    const double p = o.gx + phc;
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[0] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
    const double M1a = mfma44(P, o.a, 0.0);
    const double M1b = mfma44(P, isB ? o.bq : (isE ? o.e : 0.0), isE ? p : 0.0);
    // the next stage's operands, issued behind the first products (the
    // scheduler would otherwise sink them to their use: an LDS round trip
    // at the head of every stage)
    __builtin_amdgcn_sched_barrier(0);
    nx = load(k > 0 ? k - 1 : 0);
    __builtin_amdgcn_sched_barrier(0);
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[1] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
    const double Bz = isB ? o.bq : 0.0;
    const double AtPA = mfma44(o.a, M1a, 0.0);
    const double AtM1b = mfma44(o.a, M1b, 0.0);
    const double BtPA = mfma44(Bz, M1a, 0.0);
    const double BtM1b = mfma44(Bz, M1b, 0.0);
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[2] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
    // G = R + H2uu + Sigma_u + B'PB, h = g_u + B'Pe (block 0, lanes 0, 16, 17; 2, 18)
    double G[3], Gi[3];
    G[0] = o.wuu0 + o.su0 + dreg + lane_bcast(BtM1b, 0);
    G[1] = o.wuu1 + lane_bcast(BtM1b, 16);
    G[2] = o.wuu2 + o.su1 + dreg + lane_bcast(BtM1b, 17);
    const double h0 = o.gu0 + lane_bcast(BtM1b, 2), h1 = o.gu1 + lane_bcast(BtM1b, 18);
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[3] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
    ok = inv2(G, Gi) && ok;
    const double kk0 = -(Gi[0] * h0 + Gi[1] * h1), kk1 = -(Gi[1] * h0 + Gi[2] * h1);
    const double Hx = rowU ? BtPA + o.wxu : 0.0;
    const double mGi = (rowU && isB) ? -(r == c ? (r == 0 ? Gi[0] : Gi[2]) : Gi[1]) : 0.0;
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[4] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
    const double K = mfma44(mGi, Hx, 0.0);
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[5] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
    const double kkv = (rowU && isE) ? (r == 0 ? kk0 : kk1) : 0.0;
    Ph = mfma44(Hx, K, AtPA);
    phc = mfma44(Hx, kkv, AtM1b);
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[6] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
    if (store) {
      if (c <= r) S[oPP] = P;
      if (rowU) {
        S[oKM] = K;
        if (isE) S[L::KV + r] = kkv;
      }
      if (isE) S[L::PV + r] = p;
      if (r == 0 && c < 3) S[L::GI + c] = Gi[c];
    }
  }
    { __builtin_amdgcn_sched_barrier(0); const unsigned t_ = cyc(); seg[7] += (t_ - tprev) & 0xFFFFF; tprev = t_; __builtin_amdgcn_sched_barrier(0); }
  return ok;
}


__global__ __launch_bounds__(64, 1) void probe_seg(const double* init, long long* t) {
  __shared__ double W[N * L::F];
  for (int e = threadIdx.x; e < N * L::F; e += 64) W[e] = init[e];
  wave_lds_sync();
  unsigned seg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool ok = ric_t<L::GA + 2, L::GA, L::DXA, L::DUA>(W, N, 0.0, seg);
  if (threadIdx.x == 0) { for (int i = 0; i < 8; ++i) t[i] = seg[i]; t[8] = ok; }
}
__global__ __launch_bounds__(64, 1) void probe(const double* init, long long* t, double* out) {
  __shared__ double W[N * L::F];
  for (int e = threadIdx.x; e < N * L::F; e += 64) W[e] = init[e];
  wave_lds_sync();
  long long t0 = clock64();
  bool ok = ipmw::riccati_mfma<L::GA + 2, L::GA, L::DXA, L::DUA>(W, N, 0.0);
  wave_lds_sync();
  long long t1 = clock64();
  ipmw::forward_mfma<L::DX>(W, N);
  wave_lds_sync();
  long long t2 = clock64();
  ipmw::rhs_mfma<L::GA + 2, L::GA>(W, N);
  wave_lds_sync();
  long long t3 = clock64();
  if (threadIdx.x == 0) { t[0] = t1 - t0; t[1] = t2 - t1; t[2] = t3 - t2; t[3] = ok; }
  for (int e = threadIdx.x; e < N * L::F; e += 64) out[e] = W[e];
}
int main() {
  const int n = N * L::F;
  double* h = (double*)malloc(n * 8);
  srand(1);
  for (int e = 0; e < n; ++e) h[e] = 0.1 * ((double)rand() / RAND_MAX - 0.5);
  for (int k = 0; k < N; ++k) {  // diagonal weights and Sigma positive
    double* S = h + k * L::F;
    for (int i = 0; i < 4; ++i) { S[L::WXX + ipm::pk(i, i)] = 1.0; S[L::DXA + i] = 0.5; S[L::DA + i * 4 + i] += 1.0; }
    for (int i = 0; i < 2; ++i) { S[L::WUU + ipm::pk(i, i)] = 1.0; S[L::DUA + i] = 0.5; }
  }
  double *d, *o; long long* t; long long ht[4];
  hipMalloc(&d, n * 8); hipMalloc(&o, n * 8); hipMalloc(&t, 32);
  hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, t, o);
  hipMemcpy(ht, t, 32, hipMemcpyDeviceToHost);
  printf("N=%d cycles/stage: riccati %.0f forward %.0f rhs %.0f (ok=%lld)\n", N, ht[0] / (double)N,
         ht[1] / (double)N, ht[2] / (double)N, ht[3]);
  long long hs[9];
  hipMalloc(&t, 9 * 8);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe_seg, dim3(1), dim3(64), 0, 0, d, t);
  hipMemcpy(hs, t, 9 * 8, hipMemcpyDeviceToHost);
  const char* nm[8] = {"stage head -> P ready", "M1a,M1b issue + prefetch", "4 products issue", "G,h (readlanes)",
                       "inverse, k, Hx, -G^-1", "K issue", "Ph, ph issue", "stores"};
  long long tot = 0;
  for (int i = 0; i < 8; ++i) tot += hs[i];
  for (int i = 0; i < 8; ++i) printf("  %-28s %6.1f cycles/stage\n", nm[i], hs[i] / (double)N);
  printf("  total (SHADER_CYCLES) %.1f cycles/stage\n", tot / (double)N);
  return 0;
}
