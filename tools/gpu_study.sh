cd $GRAFT_REPO_ROOT
bash tools/pmc.sh || exit 1
timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --spp 128 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 0 --spp 16 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit 3
tail -1 gpurun_out/bench_c3.log; tail -1 gpurun_out/bench_c4.log
