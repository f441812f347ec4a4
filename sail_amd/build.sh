#!/bin/sh
# Builds libsail_hip.so for gfx950 in-tree (sail_amd/lib/). Contraction is off everywhere: the
# kernels follow the reference's f32 expression order and the bit-defined math spec (sail_math.h).
# Also builds libsail_hip_phase.so, the same library with per-phase wave timers (-DSAIL_PHASE_TIMING=1,
# tools/phase_profile.py); tests/test_gpu_parity.py checks that it renders the same bits.
set -e
cd "$(dirname "$0")"
mkdir -p lib build
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
ARCH=${SAIL_ARCH:-gfx950}
COMMON="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-unused-function"
OBJS="sail_trace sail_trace_phase sail_capi sail_hostmath sail_jit sail_jit_src"
for o in $OBJS; do rm -f build/$o.o; done  # a failed compile must not leave an older object to link
# the per-plugin-set kernels compiled at run time (sail_jit.cpp) carry the kernel sources in the library
python3 gen_jit_src.py build/sail_jit_src.cpp csrc
PIDS=""
$HIPCC $COMMON --offload-arch=$ARCH -c csrc/sail_trace.hip -o build/sail_trace.o ${SAIL_EXTRA:-} & PIDS="$PIDS $!"
$HIPCC $COMMON --offload-arch=$ARCH -DSAIL_PHASE_TIMING=1 -c csrc/sail_trace.hip -o build/sail_trace_phase.o & PIDS="$PIDS $!"
$HIPCC $COMMON --offload-arch=$ARCH -c csrc/sail_capi.cpp -o build/sail_capi.o & PIDS="$PIDS $!"
$HIPCC $COMMON --offload-arch=$ARCH -c csrc/sail_hostmath.cpp -o build/sail_hostmath.o & PIDS="$PIDS $!"
$HIPCC $COMMON --offload-arch=$ARCH -c csrc/sail_jit.cpp -o build/sail_jit.o & PIDS="$PIDS $!"
$HIPCC $COMMON --offload-arch=$ARCH -c build/sail_jit_src.cpp -o build/sail_jit_src.o & PIDS="$PIDS $!"
FAIL=0
for p in $PIDS; do wait $p || FAIL=1; done
[ $FAIL -eq 0 ] || { echo "build.sh: a compile failed"; exit 1; }
HOST="build/sail_capi.o build/sail_hostmath.o build/sail_jit.o build/sail_jit_src.o"
for o in build/sail_trace.o build/sail_trace_phase.o $HOST; do [ -s $o ] || { echo "missing $o"; exit 1; }; done
$HIPCC -shared -fPIC --offload-arch=$ARCH build/sail_trace.o $HOST -o lib/libsail_hip.so -ldl -lpthread
$HIPCC -shared -fPIC --offload-arch=$ARCH build/sail_trace_phase.o $HOST -o lib/libsail_hip_phase.so -ldl -lpthread
