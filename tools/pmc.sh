#!/bin/bash
# PMC passes for the trace kernel (one counter group per rocprofv3 run, kernel-trace only; never combined
# with sys/runtime traces). Output CSVs under gpurun_out/pmc/<pass>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p ${PMC_OUT:-gpurun_out/pmc}
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $ROOT/${PMC_OUT:-gpurun_out/pmc}/$name -o run --output-format csv -- \
    python3 $ROOT/bench.py --config ${PMC_CONFIG:-C2} --steps 1 --warmup 0 --spp ${PMC_SPP:-64} --no-cpu-baseline ${PMC_BENCH_ARGS:-} > $ROOT/${PMC_OUT:-gpurun_out/pmc}/$name.log 2>&1
}
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY || exit 1
ls $ROOT/${PMC_OUT:-gpurun_out/pmc}
