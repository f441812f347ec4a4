#!/bin/bash
# Sample-group sweep: per-rank throughput of the emulated ranks for fixed group counts (tools/scaling_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03o}
mkdir -p $OUT
for g in 1 2 4 8 16; do
  timeout -k 10 200 python -u tools/scaling_probe.py C2 1024 --groups $g --worlds 1 --reps 3 >> $OUT/g_c2.jsonl 2>&1 || exit 3
  timeout -k 10 200 python -u tools/scaling_probe.py C3 256 --groups $g --worlds 1 --reps 3 >> $OUT/g_c3.jsonl 2>&1 || exit 4
  timeout -k 10 200 python -u tools/scaling_probe.py C5 1024 --groups $g --worlds 1 --reps 3 >> $OUT/g_c5.jsonl 2>&1 || exit 5
done
for g in 8 16 32; do
  timeout -k 10 200 python -u tools/scaling_probe.py C2 1024 --groups $g --worlds 2,4,8 --reps 3 >> $OUT/g_c2n.jsonl 2>&1 || exit 6
  timeout -k 10 200 python -u tools/scaling_probe.py C3 256 --groups $g --worlds 2,4,8 --reps 3 >> $OUT/g_c3n.jsonl 2>&1 || exit 7
done
for g in 1 2 4; do
  timeout -k 10 200 python -u tools/scaling_probe.py C4 32 --groups $g --worlds 1 --reps 2 >> $OUT/g_c4.jsonl 2>&1 || exit 8
done
echo groups ok
