#!/bin/bash
# The adopted defaults (packed state per kernel set, issue priority): the whole GPU suite and smoke, the C2 bench,
# and kernel-trace summaries of the C2 bench and of the C4 wavefront split vs megakernel. Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/${SESSION_OUT:-r03h}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 3; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 4; }
timeout -k 10 400 python bench.py --no-c1-full > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 5; }
tail -1 $OUT/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_c2 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c1-full > $ROOT/$OUT/prof_c2.log 2>&1 || { tail $ROOT/$OUT/prof_c2.log; exit 6; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_c4wf -o run --output-format csv -- python3 $ROOT/bench.py --config C4 --spp 8 --launch-spp 8 --steps 1 --warmup 1 --no-cpu-baseline --wavefront > $ROOT/$OUT/prof_c4wf.log 2>&1 || { tail $ROOT/$OUT/prof_c4wf.log; exit 7; }
cd $ROOT
find $OUT -name "*kernel_stats.csv" | head -5
echo s4 ok
