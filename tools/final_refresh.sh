#!/bin/bash
# End-of-round evidence in one GPU call: tools/round_profile.sh, the VALU-mix passes, PMC summaries regenerated
# on the box (gpurun_out/summ), then the bench lines re-run so their traffic / VALU-issue fields read the fresh
# summaries, and the JS-host bench. Copy gpurun_out/summ/*.json and the bench2*.log lines into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
bash tools/round_profile.sh
PMC_OUT=gpurun_out/pmc_mix PMC_CONFIG=C2 PMC_SPP=32 bash tools/pmc_mix.sh
mkdir -p gpurun_out/summ
python tools/pmc_summary.py gpurun_out/pmc_c2 gpurun_out/summ/r01_pmc_summary.json 2073600 32 8 cornell_box_readme_C2 > /dev/null
python tools/pmc_summary.py gpurun_out/pmc_c3 gpurun_out/summ/r01_pmc_summary_c3.json 2073600 32 8 materials_demo_C3 > /dev/null
python tools/pmc_summary.py gpurun_out/pmc_c4 gpurun_out/summ/r01_pmc_summary_c4.json 8294400 32 12 random64_C4 > /dev/null
cp gpurun_out/summ/*.json profiles/
timeout -k 10 300 python bench.py > gpurun_out/bench2.log 2> gpurun_out/bench2.err
timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --spp 128 --no-cpu-baseline > gpurun_out/bench2_c3.log 2>&1
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --spp 32 --no-cpu-baseline > gpurun_out/bench2_c4.log 2>&1
timeout -k 10 300 node sail_amd/js/tools/bench_host.js > gpurun_out/bench_host.log 2>&1
tail -1 gpurun_out/bench2.log | cut -c1-200
