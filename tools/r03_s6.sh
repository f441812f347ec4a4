#!/bin/bash
# Sort skip: the GPU parity suite on the new default first (stops at the first failure), then the variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03k}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 3; }
tail -1 $OUT/pytest_gpu.log
SESSION_OUT=${SESSION_OUT:-r03k} SCENES="C1 C3 C4" bash tools/r03_variants.sh || exit 2
echo s6 ok
