bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 1 --warmup 0 --spp 64 --force-comm --no-cpu-baseline > gpurun_out/bench_comm.log 2>&1; echo "comm rc=$?"; tail -3 gpurun_out/bench_comm.log
