#!/bin/bash
# Staging as three planes with / without the first group accumulating itself: GPU suite, variants, and the
# per-rank probe at N = 1 and 8 per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03s}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 3; }
tail -1 $OUT/pytest_gpu.log
SESSION_OUT=${SESSION_OUT:-r03s} SCENES="C1 C3 C4" bash tools/r03_variants.sh > /dev/null || exit 2
for v in a_home1 b_home0; do
  for cfg in "C2 1024" "C5 1024" "C3 256"; do
    timeout -k 10 200 python -u tools/scaling_probe.py $cfg --worlds 1,8 --reps 3 --lib sail_amd/lib/variants/libsail_hip_$v.so >> $OUT/probe.jsonl 2>&1 || exit 4
  done
done
echo s9 ok
