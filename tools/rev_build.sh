#!/bin/sh
# Builds sail_amd/csrc as of git revision REV into sail_amd/lib/variants/libsail_hip_NAME.so (with its own embedded
# run-time kernel sources), the control for an A/B variant run of the working tree (tools/variant_bench.py).
# Usage: tools/rev_build.sh REV NAME
set -e
cd "$(dirname "$0")/.."
ROOT=$(pwd)
REV=$1; NAME=$2
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
COMMON="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-function --offload-arch=gfx950"
d=sail_amd/build/study/$NAME/csrc
rm -rf sail_amd/build/study/$NAME && mkdir -p $d sail_amd/lib/variants && ln -sfn ../../../include sail_amd/build/study/include
for f in $(git ls-tree --name-only $REV sail_amd/csrc/); do git show $REV:$f > $d/$(basename $f); done
git show $REV:sail_amd/gen_jit_src.py > $d/gen_jit_src.py
python3 $d/gen_jit_src.py $d/sail_jit_src.cpp $d
PIDS=""
for s in sail_trace.hip sail_capi.cpp sail_hostmath.cpp sail_jit.cpp sail_jit_src.cpp; do
  $HIPCC $COMMON -c $d/$s -o $d/${s%.*}.o & PIDS="$PIDS $!"
done
for p in $PIDS; do wait $p; done
$HIPCC -shared -fPIC --offload-arch=gfx950 $d/sail_trace.o $d/sail_capi.o $d/sail_hostmath.o $d/sail_jit.o $d/sail_jit_src.o \
  -o sail_amd/lib/variants/libsail_hip_$NAME.so -ldl -lpthread
echo "built $NAME from $REV"
