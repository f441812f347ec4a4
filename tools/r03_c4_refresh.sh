#!/bin/bash
# C4 evidence after the pre-cull kernel's shared hit-record / candidate-loop changes: rocprofv3 kernel stats of the C4
# bench, its PMC passes (summarised into gpurun_out/summ), the per-rank scaling emulation. Each GPU step has its own
# limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${FINAL_OUT:-r03c4}
mkdir -p $OUT gpurun_out/summ
ROOT=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_c4 -o run --output-format csv -- \
    python3 $ROOT/bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > $ROOT/$OUT/prof_c4.log 2>&1 ) || { tail $OUT/prof_c4.log; exit 4; }
PMC_OUT=$OUT/pmc_c4 PMC_CONFIG=C4 PMC_SPP=32 bash tools/pmc.sh > /dev/null || exit 8
python tools/pmc_summary.py $OUT/pmc_c4 gpurun_out/summ/r03_pmc_summary_c4.json 8294400 32 12 random64_C4 > /dev/null || exit 10
timeout -k 10 300 python -u tools/scaling_probe.py C4 32 > $OUT/scale_c4.jsonl 2>&1 || exit 18
echo c4 ok
