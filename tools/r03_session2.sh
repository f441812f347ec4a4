#!/bin/bash
# GPU suite on the current build (grouped pre-cull kernel of 1,024 threads + its group rule), C4 per-rank scaling
# with the new rule and forced group counts, then the variant timings. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03c}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
P="timeout -k 10 300 python -u tools/scaling_probe.py"
$P C4 32 > $OUT/scale_c4_auto.jsonl 2>&1 || { tail $OUT/scale_c4_auto.jsonl; exit 3; }
for g in 4 6 8; do $P C4 32 --groups $g --worlds 1,4,8 > $OUT/scale_c4_g$g.jsonl 2>&1 || { tail $OUT/scale_c4_g$g.jsonl; exit 4; }; done
cut -c1-200 $OUT/scale_c4_*.jsonl
SESSION_OUT=${SESSION_OUT:-r03c} SCENES="C1 C3" bash tools/r03_variants.sh || exit 5
echo session2 ok
