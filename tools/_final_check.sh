set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_gpu.log | head; exit 2; }
bash tools/r04_variants.sh cull_unroll && OUT=r04g TAG=r04 bash tools/session.sh pmc_c5
