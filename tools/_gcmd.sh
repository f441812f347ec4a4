cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -lt 2 ] && timeout -k 10 600 python tools/scaling_probe.py C2 256 > gpurun_out/scaling.log 2>&1; cat gpurun_out/scaling.log
