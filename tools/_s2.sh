set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests/test_gpu_pool.py -x -v --timeout 300 --timeout-method thread > gpurun_out/s2/pytest_pool.log 2>&1; rc=$?; tail -15 gpurun_out/s2/pytest_pool.log; [ $rc -ne 0 ] && exit 2
for cfg in C2 C3; do
  for pool in 0 1; do
    timeout -k 10 300 python bench.py --config $cfg --spp 256 --steps 3 --warmup 1 --no-cpu-baseline --debug 9=$pool > gpurun_out/s2/bench_${cfg}_$pool.log 2>&1 || exit 3
    python -c "import json,sys; d=json.loads(open('gpurun_out/s2/bench_${cfg}_$pool.log').read().strip().splitlines()[-1]); print('$cfg pool=$pool', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"
  done
done
