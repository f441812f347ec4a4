cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python tools/variant_bench.py C1 > gpurun_out/var_c1.log 2>&1; cat gpurun_out/var_c*.log
