#!/bin/bash
# Round-6 study session (through gpurun): variant timings with bit-identity checks, then PMC passes of chosen counters on
# the product and on variants. Each GPU step under its own time limit; stops at the first failure.
#   OUT=r06b STUDY_SCENES="C1 C3 C4" STUDY_VARIANTS="rank_wave" PMC_SETS="lds" bash tools/r06_studies.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/${OUT:-r06s}
mkdir -p $OUT
specs="main=main"
for v in ${STUDY_VARIANTS:-}; do specs="$specs $v=sail_amd/lib/variants/libsail_hip_$v.so"; done
for sc in ${STUDY_SCENES:-C1}; do
  echo "== variants $sc"
  VARIANT_ROUNDS=${VARIANT_ROUNDS:-2} timeout -k 10 ${VARIANT_TIMEOUT:-600} python -u tools/variant_bench.py $sc $specs \
    > $OUT/variants_$sc.jsonl 2> $OUT/variants_$sc.err || { tail $OUT/variants_$sc.err; exit 2; }
  cat $OUT/variants_$sc.jsonl
done
declare -A SETS=(
  [lds]="SQ_INSTS_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
  [core]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  [wait]="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_INSTS_BRANCH"
)
cd /tmp && export TMPDIR=/tmp
for set in ${PMC_SETS:-}; do
  for v in main ${PMC_VARIANTS:-${STUDY_VARIANTS:-}}; do
    for cfg in ${PMC_CONFIGS:-C2}; do
      lib=""; [ $v != main ] && lib=$ROOT/sail_amd/lib/variants/libsail_hip_$v.so
      spp=64; [ $cfg = C2 ] && spp=1024
      echo "== pmc $set $v $cfg"
      SAIL_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --pmc ${SETS[$set]} -d $ROOT/$OUT/pmc_${set}_${v}_$cfg -o run --output-format csv -- \
        python3 $ROOT/bench.py --config $cfg --steps 1 --warmup 0 --spp $spp --no-cpu-baseline --no-validate \
        > $ROOT/$OUT/pmc_${set}_${v}_$cfg.log 2>&1 || { tail -5 $ROOT/$OUT/pmc_${set}_${v}_$cfg.log; exit 3; }
      python3 - $ROOT/$OUT/pmc_${set}_${v}_$cfg <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "sail_trace_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: sum(v) / len(v) for k, v in sorted(agg.items())})
PY
    done
  done
done
echo "studies ok"
