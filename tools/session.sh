#!/bin/bash
# One GPU session (run through gpurun): the named steps in order, each GPU step under its own time limit; the script
# stops at the first failure, so nothing touches the GPU after a crash, abort or timeout. Output under gpurun_out/$OUT.
#   OUT=r04a bash tools/session.sh tests smoke bench prof_c2 pmc_c3 ...
# Steps:
#   tests            pytest -m gpu (the driver's suite)              smoke       __graft_entry__.smoke()
#   bench            bench.py C2 with the CPU baselines               bench_quick bench.py C2, no CPU baseline
#   bench_c3|c4|c5   the config's full frame                          bench_rccl  C2 through the forced-RCCL branch
#   prof_c2|c3|c4|c5 rocprofv3 --kernel-trace --stats of the config's bench (C4 at 64 spp: one launch)
#   pmc_c2|c3|c4|c5  the four PMC passes of tools/pmc.sh over one launch of the bench's shape, summarised into
#                    gpurun_out/summ/$TAG_pmc_summary_<cfg>.json
#   mix_c2|c3|c4     the VALU instruction-mix passes of tools/pmc_mix.sh, summarised the same way and paired with
#                    the pmc_<cfg> summary of the same session (refused unless both counted the same build)
#   scale            the per-rank emulation of N = 1/2/4/8 (tools/scaling_probe.py) for C2..C5
#   variants         tools/variant_bench.py over sail_amd/lib/variants/*.so (VARIANT_ARGS: scene W H B spp ...)
#   phases           tools/phase_profile.py with the phase-timing build (sail_amd/lib/libsail_hip_phase.so)
#   jshost           the JS host bench (sail_amd/js/tools/bench_host.js)
#   torchrun         bench.py under torch.distributed.run at N = 1
#   jit_times        the run-time kernels' build latency per form, cold and warm disk cache
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/${OUT:-session}
TAG=${TAG:-r04}
mkdir -p $OUT gpurun_out/summ
declare -A PX=([c2]=2073600 [c3]=2073600 [c4]=8294400 [c5]=2073600)
declare -A BO=([c2]=8 [c3]=8 [c4]=12 [c5]=16)
declare -A WL=([c2]=cornell_box_readme_C2 [c3]=materials_demo_C3 [c4]=random64_C4 [c5]=cornell_box_converged_C5)
declare -A OPS=([c2]=298.98 [c3]=889.32 [c4]=4061.12 [c5]=296.66)
# samples of the one profiled launch: the bench's own launch shape (the Cornell form runs 1,024 samples per launch)
declare -A LS=([c2]=1024 [c3]=64 [c4]=64 [c5]=1024)
prof() {  # rocprofv3 kernel stats of a bench run: prof <name> <bench args...>
  local name=$1; shift
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/$name -o run \
      --output-format csv -- python3 $ROOT/bench.py "$@" > $ROOT/$OUT/$name.log 2>&1 )
}
for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit 2 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
      cat $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.log 2> $OUT/bench.err || { tail $OUT/bench.err; exit 4; }
      cut -c1-400 $OUT/bench.log ;;
    bench_quick)
      timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_quick.log 2> $OUT/bench_quick.err || { tail $OUT/bench_quick.err; exit 4; }
      cut -c1-400 $OUT/bench_quick.log ;;
    bench_rccl)
      timeout -k 10 300 python bench.py --force-rccl --no-cpu-baseline > $OUT/bench_rccl.log 2> $OUT/bench_rccl.err || { tail $OUT/bench_rccl.err; exit 4; }
      cut -c1-300 $OUT/bench_rccl.log ;;
    bench_c3|bench_c4|bench_c5)
      cfg=$(echo ${step#bench_} | tr a-z A-Z)
      timeout -k 10 400 python bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline > $OUT/$step.log 2> $OUT/$step.err || { tail $OUT/$step.err; exit 5; }
      cut -c1-400 $OUT/$step.log ;;
    prof_c2) prof prof_c2 --steps 3 --warmup 1 --no-cpu-baseline || exit 6 ;;
    prof_c3) prof prof_c3 --config C3 --steps 1 --warmup 1 --no-cpu-baseline || exit 6 ;;
    prof_c4) prof prof_c4 --config C4 --steps 1 --warmup 1 --spp 64 --no-cpu-baseline || exit 6 ;;
    prof_c5) prof prof_c5 --config C5 --steps 1 --warmup 1 --no-cpu-baseline || exit 6 ;;
    pmc_c2|pmc_c3|pmc_c4|pmc_c5)
      c=${step#pmc_}; cfg=$(echo $c | tr a-z A-Z)
      PMC_OUT=$OUT/$step PMC_CONFIG=$cfg PMC_SPP=${LS[$c]} bash tools/pmc.sh > /dev/null || exit 7  # one launch
      python tools/pmc_summary.py $OUT/$step gpurun_out/summ/${TAG}_pmc_summary_$c.json ${PX[$c]} ${LS[$c]} ${BO[$c]} ${WL[$c]} > /dev/null || exit 7 ;;
    mix_c2|mix_c3|mix_c4)
      c=${step#mix_}; cfg=$(echo $c | tr a-z A-Z)
      PMC_OUT=$OUT/$step PMC_CONFIG=$cfg PMC_SPP=${LS[$c]} bash tools/pmc_mix.sh > /dev/null || exit 8
      # paired with this session's PMC summary of the same config (run pmc_<cfg> first): refused unless the same build
      python tools/pmc_mix_summary.py $OUT/$step gpurun_out/summ/${TAG}_pmc_valu_mix_$c.json ${PX[$c]} ${LS[$c]} ${BO[$c]} ${WL[$c]} ${OPS[$c]} \
        gpurun_out/summ/${TAG}_pmc_summary_$c.json > /dev/null || exit 8 ;;
    scale)
      for a in "C2 1024" "C3 256" "C4 32" "C5 1024"; do
        timeout -k 10 300 python -u tools/scaling_probe.py $a >> $OUT/scale.jsonl 2>&1 || exit 9
      done ;;
    variants)
      timeout -k 10 900 python -u tools/variant_bench.py ${VARIANT_ARGS:-} > $OUT/variants.jsonl 2> $OUT/variants.err || { tail $OUT/variants.err; exit 10; }
      cat $OUT/variants.jsonl ;;
    phases)
      timeout -k 10 600 python -u tools/phase_profile.py sail_amd/lib/libsail_hip_phase.so ${PHASE_SCENES:-C1 C3 C4} > $OUT/phases.jsonl 2>&1 || { tail $OUT/phases.jsonl; exit 11; }
      cat $OUT/phases.jsonl ;;
    torchrun)  # bench.py under torch.distributed.run at N = 1 (the launcher the driver uses for N > 1)
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_torchrun.log \
        2> $OUT/bench_torchrun.err || { tail $OUT/bench_torchrun.err; exit 13; }
      cut -c1-300 $OUT/bench_torchrun.log ;;
    jit_times)  # run-time kernel build latency per form, cold and warm (tools/jit_compile_times.py)
      timeout -k 10 900 python -u tools/jit_compile_times.py > $OUT/jit_compile_times.jsonl 2> $OUT/jit_compile_times.err || { tail $OUT/jit_compile_times.err; exit 14; }
      cat $OUT/jit_compile_times.jsonl ;;
    jshost)
      timeout -k 10 300 node sail_amd/js/tools/bench_host.js > $OUT/bench_js_host.json 2> $OUT/bench_js_host.err || exit 12
      cut -c1-300 $OUT/bench_js_host.json ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "session ok"
