#!/bin/bash
# Re-entry session evidence for the pre-cull kernel's two-barrier sort: parity suite + smoke, C4 bench lines
# (32 spp and the full 256 spp), rocprofv3 kernel stats of the 32-spp line, the C4 PMC summary, then the C2 bench.
# Every GPU step has its own limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02e
mkdir -p $OUT gpurun_out/summ
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || exit 4
tail -1 $OUT/bench_c4.log | cut -c1-200
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c4_full.log 2>&1 || exit 5
tail -1 $OUT/bench_c4_full.log | cut -c1-200
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_c4 -o run --output-format csv -- \
    python3 $ROOT/bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > $ROOT/$OUT/prof_c4.log 2>&1 ) || { tail $OUT/prof_c4.log; exit 6; }
PMC_OUT=$OUT/pmc_c4 PMC_CONFIG=C4 PMC_SPP=32 bash tools/pmc.sh > /dev/null || exit 7
python tools/pmc_summary.py $OUT/pmc_c4 gpurun_out/summ/r02_pmc_summary_c4.json 8294400 32 12 random64_C4 > /dev/null || exit 8
timeout -k 10 400 python bench.py > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 9; }
tail -1 $OUT/bench.log | cut -c1-200
echo r02e ok
