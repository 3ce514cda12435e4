#!/bin/bash
# A/B variant of libmpcqp.so: recompile the given sources with extra flags and
# link them with the product objects (make first).  In the container:
#   bash tools/ab_build.sh TAG "-DFLAG=1" quad_box.hip [more.hip ...]
# -> model_predictive_control_amd/lib/variants/libmpcqp_TAG.so (select it on
# the GPU box with MPCQP_LIB=...).
set -e
TAG=$1; FLAGS=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/model_predictive_control_amd/csrc
OBJ=$ROOT/model_predictive_control_amd/lib/obj
OUT=$ROOT/model_predictive_control_amd/lib/variants
mkdir -p $OUT/obj_$TAG
objs=()
for o in $OBJ/*.o; do
  base=$(basename $o .o)
  if printf '%s\n' "$@" | grep -qx "$base"; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
      -munsafe-fp-atomics -I$ROOT/include $FLAGS -c $CS/$base -o $OUT/obj_$TAG/$base.o &
    objs+=($OUT/obj_$TAG/$base.o)
  else
    objs+=($o)
  fi
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libmpcqp_$TAG.so "${objs[@]}"
rm -rf $OUT/obj_$TAG
echo "built $OUT/libmpcqp_$TAG.so"
