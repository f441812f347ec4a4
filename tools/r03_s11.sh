#!/bin/bash
# The general square root by the corrected hardware root: exhaustive probe first, then the GPU suite, then variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03ag}
mkdir -p $OUT
timeout -k 10 120 ./sail_amd/build/sqrt01_probe > $OUT/sqrt_probe.json 2>&1 || { cat $OUT/sqrt_probe.json; exit 2; }
cat $OUT/sqrt_probe.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 3; }
tail -1 $OUT/pytest_gpu.log
SESSION_OUT=${SESSION_OUT:-r03ag} SCENES="C1 C3 C4" bash tools/r03_variants.sh > /dev/null || exit 4
cut -c1-150 $OUT/variants.log
echo s11 ok
