#!/bin/sh
# Builds experimental variants of libsail_hip.so (same sources, different -D flags) into sail_amd/lib/variants/.
# Usage: tools/build_variants.sh name1 "-DFLAG=1" name2 "-DFLAG=2" ...
# A flags string may start with "src=<file under csrc/>" to build that source instead of sail_trace.hip.
set -e
cd "$(dirname "$0")/../sail_amd"
mkdir -p lib/variants build/variants
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
COMMON="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-function --offload-arch=gfx950"
$HIPCC $COMMON -c csrc/sail_capi.cpp -o build/variants/sail_capi.o
$HIPCC $COMMON -c csrc/sail_hostmath.cpp -o build/variants/sail_hostmath.o
python3 gen_jit_src.py build/variants/sail_jit_src.cpp csrc
$HIPCC $COMMON -c csrc/sail_jit.cpp -o build/variants/sail_jit.o
$HIPCC $COMMON -c build/variants/sail_jit_src.cpp -o build/variants/sail_jit_src.o
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  src=sail_trace.hip
  case "$flags" in src=*) src=${flags%% *}; src=${src#src=}; flags=${flags#src=$src}; esac
  $HIPCC $COMMON $flags -Icsrc -c csrc/$src -o build/variants/trace_$name.o
  $HIPCC -shared -fPIC --offload-arch=gfx950 build/variants/trace_$name.o build/variants/sail_capi.o \
    build/variants/sail_hostmath.o build/variants/sail_jit.o build/variants/sail_jit_src.o -o lib/variants/libsail_hip_$name.so -ldl
  echo "built $name ($flags)"
done
