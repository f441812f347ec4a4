#!/bin/sh
# Study builds: a copy of sail_amd/csrc patched by tools/study.py <name> (string replacements catalogued in tools/studies.json), built
# like the product into sail_amd/lib/variants/libsail_hip_<name>.so. The product sources are never edited; results of
# a study are measured by tools/variant_bench.py and recorded in profiles/.
# Usage: tools/study_build.sh name [name ...]
set -e
cd "$(dirname "$0")/.."
ROOT=$(pwd)
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
COMMON="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-function --offload-arch=gfx950"
mkdir -p sail_amd/lib/variants
for name in "$@"; do
  d=sail_amd/build/study/$name/csrc   # two levels below the root, like sail_amd/csrc: "../../include" resolves
  rm -rf sail_amd/build/study/$name && mkdir -p $d && cp sail_amd/csrc/* $d/ && ln -sfn ../../../include sail_amd/build/study/include
  python3 tools/study.py $name $d
  $HIPCC $COMMON -c $d/sail_trace.hip -o $d/sail_trace.o &
  $HIPCC $COMMON -c $d/sail_capi.cpp -o $d/sail_capi.o &
  $HIPCC $COMMON -c $d/sail_hostmath.cpp -o $d/sail_hostmath.o &
  python3 sail_amd/gen_jit_src.py $d/sail_jit_src.cpp $d
  $HIPCC $COMMON -c $d/sail_jit.cpp -o $d/sail_jit.o &
  $HIPCC $COMMON -c $d/sail_jit_src.cpp -o $d/sail_jit_src.o &
  wait
  for o in sail_trace sail_capi sail_hostmath sail_jit sail_jit_src; do [ -s $d/$o.o ] || { echo "study $name: $o failed"; exit 1; }; done
  $HIPCC -shared -fPIC --offload-arch=gfx950 $d/sail_trace.o $d/sail_capi.o $d/sail_hostmath.o $d/sail_jit.o \
    $d/sail_jit_src.o -o sail_amd/lib/variants/libsail_hip_$name.so -ldl
  echo "built $name"
done
