#!/bin/bash
# Occupancy vs spill-traffic sweep of one trace kernel (run on the GPU box after tools/build_variants.sh has built
# sail_amd/lib/variants/libsail_hip_<name>.so): per variant, the C4 (or $OCC_SCENE) render time (tools/debug_bench.py,
# bit-identity checked) and the HBM bytes of its launches (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, one counter
# group per run, kernel trace only). Output: gpurun_out/occ/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/occ
mkdir -p $OUT
SCENE=${OCC_SCENE:-C4}
for so in sail_amd/lib/variants/libsail_hip_*.so; do
  v=$(basename $so .so); v=${v#libsail_hip_}
  timeout -k 10 300 python tools/debug_bench.py --lib $so $SCENE > $OUT/${v}_time.log 2>&1 || { cat $OUT/${v}_time.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $c -d $OUT/${v}_$c -o run --output-format csv -- \
        python3 $ROOT/tools/debug_bench.py --lib $ROOT/$so $SCENE > $OUT/${v}_$c.log 2>&1 ) || { tail $OUT/${v}_$c.log; exit 2; }
  done
  cat $OUT/${v}_time.log
done
