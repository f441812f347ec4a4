#!/bin/bash
# Round-3 evidence in one GPU call: parity suite + smoke; rocprofv3 kernel stats of the C2 and C4 benches; PMC
# passes for C2/C3/C4 (one counter group per run, kernel-trace only) summarised on the box into
# gpurun_out/summ/r03_*.json and copied into profiles/ there; the C3 VALU mix; then the bench lines (C2 with the CPU
# baselines, C2 through the forced-RCCL multi-device branch, C3/C4/C5 in full) so their traffic / VALU-issue fields
# read the fresh summaries; the per-rank scaling emulation; the JS-host bench. Every GPU step has its own limit;
# the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${FINAL_OUT:-r03final}
mkdir -p $OUT gpurun_out/summ
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c1-full > $ROOT/$OUT/prof.log 2>&1 ) || { tail $OUT/prof.log; exit 4; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_c4 -o run --output-format csv -- \
    python3 $ROOT/bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > $ROOT/$OUT/prof_c4.log 2>&1 ) || { tail $OUT/prof_c4.log; exit 5; }
PMC_OUT=$OUT/pmc_c2 PMC_CONFIG=C2 PMC_SPP=64 bash tools/pmc.sh > /dev/null || exit 6
PMC_OUT=$OUT/pmc_c3 PMC_CONFIG=C3 PMC_SPP=64 bash tools/pmc.sh > /dev/null || exit 7
PMC_OUT=$OUT/pmc_c4 PMC_CONFIG=C4 PMC_SPP=32 bash tools/pmc.sh > /dev/null || exit 8
PMC_OUT=$OUT/pmc_mix_c3 PMC_CONFIG=C3 PMC_SPP=32 bash tools/pmc_mix.sh > /dev/null || exit 9
python tools/pmc_summary.py $OUT/pmc_c2 gpurun_out/summ/r03_pmc_summary.json 2073600 32 8 cornell_box_readme_C2 > /dev/null || exit 10
python tools/pmc_summary.py $OUT/pmc_c3 gpurun_out/summ/r03_pmc_summary_c3.json 2073600 32 8 materials_demo_C3 > /dev/null || exit 10
python tools/pmc_summary.py $OUT/pmc_c4 gpurun_out/summ/r03_pmc_summary_c4.json 8294400 32 12 random64_C4 > /dev/null || exit 10
python tools/pmc_mix_summary.py $OUT/pmc_mix_c3 gpurun_out/summ/r03_pmc_valu_mix_c3.json 2073600 32 8 materials_demo_C3 889.32 > /dev/null || exit 10
cp gpurun_out/summ/r03_*.json profiles/
timeout -k 10 400 python bench.py > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 11; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 python bench.py --force-rccl --no-cpu-baseline --no-c1-full > $OUT/bench_rccl1.log 2> $OUT/bench_rccl1.err || { tail $OUT/bench_rccl1.err; exit 12; }
timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c3_full.log 2>&1 || exit 13
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c4_full.log 2>&1 || exit 14
timeout -k 10 300 python bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_c5_full.log 2>&1 || exit 15
for f in bench_rccl1 bench_c3_full bench_c4_full bench_c5_full; do tail -1 $OUT/$f.log | cut -c1-200; done
timeout -k 10 300 python -u tools/scaling_probe.py C2 1024 > $OUT/scale_c2.jsonl 2>&1 || exit 16
timeout -k 10 300 python -u tools/scaling_probe.py C3 256 > $OUT/scale_c3.jsonl 2>&1 || exit 17
timeout -k 10 300 python -u tools/scaling_probe.py C4 32 > $OUT/scale_c4.jsonl 2>&1 || exit 18
timeout -k 10 300 python -u tools/scaling_probe.py C5 1024 > $OUT/scale_c5.jsonl 2>&1 || exit 19
timeout -k 10 300 node sail_amd/js/tools/bench_host.js > $OUT/bench_js_host.json 2> $OUT/bench_js_host.err || exit 20
cut -c1-300 $OUT/bench_js_host.json
echo final ok
