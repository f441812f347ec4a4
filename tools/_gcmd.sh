cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -lt 2 ] && \
timeout -k 10 600 python bench.py --config C5 --spp 256 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1; tail -1 gpurun_out/bench_c5.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['filter'])"
