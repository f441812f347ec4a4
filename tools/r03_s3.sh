#!/bin/bash
# Packed-state variants, the wavefront split's parity tests, and the wavefront split vs the megakernel on C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03g}
mkdir -p $OUT
SESSION_OUT=${SESSION_OUT:-r03g} SCENES="C1 C3 C4" bash tools/r03_variants.sh || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wavefront or precull_sample_groups" > $OUT/pytest_wf.log 2>&1 || { tail -30 $OUT/pytest_wf.log; exit 3; }
tail -1 $OUT/pytest_wf.log
timeout -k 10 300 python bench.py --config C4 --spp 8 --launch-spp 8 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c4_mega8.log 2>&1 || { tail $OUT/bench_c4_mega8.log; exit 4; }
timeout -k 10 300 python bench.py --config C4 --spp 8 --launch-spp 8 --steps 1 --warmup 1 --no-cpu-baseline --wavefront > $OUT/bench_c4_wf8.log 2>&1 || { tail $OUT/bench_c4_wf8.log; exit 5; }
tail -1 $OUT/bench_c4_mega8.log | cut -c1-200; tail -1 $OUT/bench_c4_wf8.log | cut -c1-200
echo s3 ok
