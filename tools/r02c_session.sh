#!/bin/bash
# Round-2 (third part) evidence for the pre-cull kernel: parity suite on the current build, C4 PMC passes and
# summary, rocprofv3 kernel stats of the C4 bench, and the C3/C4 bench lines at 32 spp and at their configs' own spp
# (C3 1024, C4 256). Every GPU step has its own limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02c
mkdir -p $OUT gpurun_out/summ
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
PMC_OUT=$OUT/pmc_c4 PMC_CONFIG=C4 PMC_SPP=32 bash tools/pmc.sh > /dev/null || exit 5
python tools/pmc_summary.py $OUT/pmc_c4 gpurun_out/summ/r02_pmc_summary_c4.json 8294400 32 12 random64_C4 > /dev/null || exit 6
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_c4 -o run --output-format csv -- \
    python3 $ROOT/bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > $ROOT/$OUT/prof_c4.log 2>&1 ) || { tail $OUT/prof_c4.log; exit 4; }
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c4_full.log 2>&1 || exit 12
timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --spp 128 --no-cpu-baseline > $OUT/bench_c3.log 2>&1 || exit 13
timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c3_full.log 2>&1 || exit 14
for f in bench_c4 bench_c4_full bench_c3 bench_c3_full; do tail -1 $OUT/$f.log | cut -c1-220; done
echo r02c ok
