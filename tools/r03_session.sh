#!/bin/bash
# Round-3 first GPU call: the new checkpoint / queue / forced-RCCL tests first, then the whole GPU suite and smoke,
# the C2 bench (with its post-timing frame validation), the multi-device RCCL path at one GPU through the bench,
# and the JS-host bench (per-frame renders now batched). Every GPU step has its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03a}
mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_checkpoint.py tests/test_gpu_multi.py -m gpu > $OUT/pytest_new.log 2>&1 || { tail -30 $OUT/pytest_new.log; exit 2; }
tail -1 $OUT/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 3; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 4; }
timeout -k 10 400 python bench.py --no-c1-full > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 5; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --force-rccl --no-cpu-baseline > $OUT/bench_rccl1.log 2> $OUT/bench_rccl1.err || { tail $OUT/bench_rccl1.err; exit 6; }
tail -1 $OUT/bench_rccl1.log | cut -c1-300
timeout -k 10 300 node sail_amd/js/tools/bench_host.js > $OUT/bench_js_host.json 2> $OUT/bench_js_host.err || { cat $OUT/bench_js_host.err; exit 7; }
cut -c1-400 $OUT/bench_js_host.json
echo session ok
