#!/bin/sh
# AddressSanitizer + UndefinedBehaviorSanitizer builds of the HOST code, for tests/test_sanitizers.py:
#   build/sanitize/libsail_hip_asan.so  sail_capi.cpp + sail_hostmath.cpp instrumented (-fno-gpu-sanitize: the
#                                       device code is the product's own sail_trace.o, never instrumented)
#   build/sanitize/libsail_oracle_asan.so  the CPU oracle
#   build/sanitize/sail_napi_asan.node  the Node-API addon, linked to the instrumented library
# All use clang's shared ASan runtime (one runtime per process; the test preloads it into python / node).
set -e
cd "$(dirname "$0")/.."
OUT=build/sanitize
mkdir -p $OUT
CLANG=/opt/rocm/lib/llvm/bin/clang++
HIPCC=/opt/rocm/bin/hipcc
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -shared-libasan -g -O1"
[ -f sail_amd/build/sail_trace.o ] || sh sail_amd/build.sh
for f in sail_capi sail_hostmath sail_jit; do
  $HIPCC -std=c++17 -fPIC -ffp-contract=off -fno-fast-math $SAN -fno-gpu-sanitize --offload-arch=gfx950 \
    -c sail_amd/csrc/$f.cpp -o $OUT/$f.o
done
$HIPCC -shared -fPIC -shared-libasan -fsanitize=address,undefined -fno-gpu-sanitize --offload-arch=gfx950 \
  sail_amd/build/sail_trace.o $OUT/sail_capi.o $OUT/sail_hostmath.o $OUT/sail_jit.o sail_amd/build/sail_jit_src.o \
  -o $OUT/libsail_hip_asan.so -ldl
$CLANG -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math $SAN oracle/sail_oracle.cpp \
  -o $OUT/libsail_oracle_asan.so
if [ -d /usr/include/node ]; then
  # (globals not instrumented in the addon: at require() its string-literal globals were registered twice, an
  # ODR false positive that aborts the run)
  $CLANG -std=c++17 -fPIC -shared $SAN -mllvm -asan-globals=0 -DNODE_GYP_MODULE_NAME=sail_napi -DNAPI_VERSION=8 -I/usr/include/node \
    sail_amd/js/native/sail_napi.cc -o $OUT/sail_napi_asan.node -L$OUT -lsail_hip_asan -Wl,-rpath,"$(pwd)/$OUT"
fi
echo "sanitized builds in $OUT"
