#!/bin/bash
# The new sample-group rule (auto) at N = 1/2/4/8 for every config, and the pre-cull kernel's target swept.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03p}
mkdir -p $OUT
timeout -k 10 300 python -u tools/scaling_probe.py C2 1024 --reps 3 >> $OUT/auto.jsonl 2>&1 || exit 3
timeout -k 10 300 python -u tools/scaling_probe.py C3 256 --reps 3 >> $OUT/auto.jsonl 2>&1 || exit 4
timeout -k 10 300 python -u tools/scaling_probe.py C4 32 --reps 2 >> $OUT/auto.jsonl 2>&1 || exit 5
timeout -k 10 300 python -u tools/scaling_probe.py C5 1024 --reps 3 >> $OUT/auto.jsonl 2>&1 || exit 6
for r in 16 32 128; do
  timeout -k 10 300 python -u tools/scaling_probe.py C4 32 --reps 2 --cull-rounds $r >> $OUT/cull_rounds.jsonl 2>&1 || exit 7
done
for r in 18 72; do
  timeout -k 10 300 python -u tools/scaling_probe.py C2 1024 --reps 3 --rounds $r >> $OUT/flat_rounds.jsonl 2>&1 || exit 8
done
echo groups2 ok
