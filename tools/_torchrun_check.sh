set -o pipefail
mkdir -p gpurun_out/r04i
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04i/bench_torchrun.log 2> gpurun_out/r04i/bench_torchrun.err || { tail gpurun_out/r04i/bench_torchrun.err; exit 2; }
cut -c1-300 gpurun_out/r04i/bench_torchrun.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04i/smoke.log 2>&1 || { cat gpurun_out/r04i/smoke.log; exit 3; }
cat gpurun_out/r04i/smoke.log
