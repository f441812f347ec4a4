#!/bin/bash
# VALU instruction-mix PMC passes for the trace kernel (two runs of 8 SQ counters each; kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=${PMC_OUT:-gpurun_out/pmc_mix}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $ROOT/$OUT/$name -o run --output-format csv -- \
    python3 $ROOT/bench.py --config ${PMC_CONFIG:-C2} --steps 1 --warmup 0 --spp ${PMC_SPP:-64} --no-cpu-baseline ${PMC_BENCH_ARGS:-} > $ROOT/$OUT/$name.log 2>&1
}
run mix1 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 || exit 1
run mix2 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_INT64 SQ_WAVES SQ_BUSY_CYCLES || exit 1
