#!/bin/bash
# One call, several steps (calls rarely reach a box at the moment): variant timings, the GPU suite on the current
# build, C4 per-rank scaling with the current group rule, the C2 bench. Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03f}
mkdir -p $OUT
SESSION_OUT=${SESSION_OUT:-r03f} SCENES="C1 C3 C4" bash tools/r03_variants.sh || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 3; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/scaling_probe.py C4 32 > $OUT/scale_c4_auto.jsonl 2>&1 || { tail $OUT/scale_c4_auto.jsonl; exit 4; }
cut -c1-200 $OUT/scale_c4_auto.jsonl
timeout -k 10 400 python bench.py --no-c1-full > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 5; }
tail -1 $OUT/bench.log | cut -c1-300
echo big ok
