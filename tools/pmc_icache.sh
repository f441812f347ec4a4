#!/bin/bash
# Instruction-cache / issue-wait PMC pass (PMC_SET=icache) or LDS / scalar-memory pass (PMC_SET=lds) for the
# trace kernel of each workload (one run of 8 SQ counters per config; kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=${PMC_OUT:-gpurun_out/pmc_icache}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for cfg in ${PMC_CONFIGS:-C2 C3 C4}; do
  if [ "${PMC_SET:-icache}" = lds ]; then
    set -- SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE \
      SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
  else
    set -- SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY \
      SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU
  fi
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $ROOT/$OUT/$cfg -o run --output-format csv -- \
    python3 $ROOT/bench.py --config $cfg --steps 1 --warmup 0 --spp 32 --no-cpu-baseline > $ROOT/$OUT/$cfg.log 2>&1 || exit 1
done
