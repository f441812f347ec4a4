#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace of the bench.
# Each GPU step has its own time limit; a crash/abort/timeout (exit >= 2 from pytest, or any non-zero
# from the other steps) ends the script before anything else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
STEPS=${BENCH_STEPS:-2}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a $OUT/pytest_gpu.log
tail -5 $OUT/pytest_gpu.log
if [ $rc -ge 2 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 3; }
cat $OUT/smoke.log
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 > $OUT/bench.log 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 4; }
cat $OUT/bench.log
[ "${SKIP_PROF:-0}" = "1" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 5; }
find $GRAFT_REPO_ROOT/$OUT/prof -name "*stats*" | head
