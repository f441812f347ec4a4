#!/bin/bash
# One GPU session producing the round's evidence: parity suite, C2 bench (with CPU baseline), rocprofv3
# kernel stats of the C2 bench, C3/C4 bench lines, PMC passes for C2/C3/C4. Every GPU step has its own time
# limit and the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 4; }
timeout -k 10 600 python bench.py --config C3 --steps 1 --warmup 1 --spp 128 --no-cpu-baseline > $OUT/bench_c3.log 2>&1 || exit 5
timeout -k 10 600 python bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || exit 6
ROOT=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $ROOT/$OUT/prof.log 2>&1 ) || exit 7
PMC_OUT=$OUT/pmc_c2 PMC_CONFIG=C2 bash tools/pmc.sh || exit 8
PMC_OUT=$OUT/pmc_c3 PMC_CONFIG=C3 bash tools/pmc.sh || exit 9
PMC_OUT=$OUT/pmc_c4 PMC_CONFIG=C4 PMC_SPP=32 bash tools/pmc.sh || exit 10
tail -1 $OUT/bench.log | cut -c1-300
