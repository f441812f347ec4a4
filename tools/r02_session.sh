#!/bin/bash
# Round-2 GPU session: parity suite, C2 bench (with the CPU baselines incl. C1 in full), the C5 converged render at
# its full 65,536 spp, and a rocprofv3 kernel trace of the C2 bench. Each GPU step has its own limit; stop at the
# first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 4; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_c5_full.log 2> $OUT/bench_c5.err || { tail $OUT/bench_c5.err; exit 5; }
tail -1 $OUT/bench_c5_full.log | cut -c1-300
ROOT=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/$OUT/prof.log 2>&1 ) || exit 6
echo session ok
