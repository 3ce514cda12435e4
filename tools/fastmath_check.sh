#!/bin/bash
# What the FASTDIV flags of csrc/Makefile (-fapprox-func -freciprocal-math)
# change in the gfx950 code, by compiling probes with and without them:
#   fp64: division only (rcp + Newton instead of div_scale/div_fmas/div_fixup);
#         sqrt, sincos, atan and tan compile to identical instruction streams
#   fp32: division (v_rcp_f32) and sqrt (v_sqrt_f32 / v_rsq_f32 without the
#         correction steps) -- used only by the MFMA sweep's 1/sqrt pivots,
#         whose results the fp64 refinement from the dynamics certifies
# Usage: bash tools/fastmath_check.sh   (CPU only; prints one line per probe)
set -euo pipefail
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
d=$(mktemp -d)
trap 'rm -rf "$d"' EXIT
cat > "$d/f64.hip" <<'EOF'
#include <hip/hip_runtime.h>
__global__ void k(const double* a, double* s, double* t) {
  const int i = threadIdx.x;
  s[i] = sqrt(a[i]);
  double sn, cs;
  sincos(a[i], &sn, &cs);
  t[i] = sn + atan(cs) + tan(a[i]) + atan(a[i] * tan(cs));
}
EOF
cat > "$d/div64.hip" <<'EOF'
#include <hip/hip_runtime.h>
__global__ void k(const double* a, const double* b, double* c) { c[threadIdx.x] = a[threadIdx.x] / b[threadIdx.x]; }
EOF
cat > "$d/f32.hip" <<'EOF'
#include <hip/hip_runtime.h>
__global__ void k(const float* a, float* s, float* t) { s[threadIdx.x] = sqrtf(a[threadIdx.x]); t[threadIdx.x] = 1.f / sqrtf(a[threadIdx.x]); }
EOF
ops() { grep -E '^\s+[vs]_' "$1" | awk '{print $1}'; }
for p in f64 div64 f32; do
  "$HIPCC" -O3 --offload-arch=gfx950 --cuda-device-only -S "$d/$p.hip" -o "$d/$p.ieee.s"
  "$HIPCC" -O3 --offload-arch=gfx950 --cuda-device-only -S -fapprox-func -freciprocal-math "$d/$p.hip" -o "$d/$p.fast.s"
  if diff -q <(ops "$d/$p.ieee.s") <(ops "$d/$p.fast.s") > /dev/null; then
    echo "$p: identical instruction stream"
  else
    echo "$p: differs -- ieee: $(ops "$d/$p.ieee.s" | grep -cE 'div|rcp|sqrt|rsq') div/rcp/sqrt ops," \
         "fast: $(ops "$d/$p.fast.s" | grep -cE 'div|rcp|sqrt|rsq')"
  fi
done
