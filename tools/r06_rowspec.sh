#!/bin/bash
# Round-6 studies: per-row specialised room form (SAIL_DEBUG_JIT bits 32 / 64) and the packed-bounds mask build
# (variant cull_b4), timed against the product with bit-identity checks (tools/variant_bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r06c}; mkdir -p $OUT
for sc in C3 UI ALL AREA; do
  VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py $sc main=main "big=main:9=59" "all=main:9=123" > $OUT/rowspec_$sc.jsonl 2> $OUT/rowspec_$sc.err || { tail $OUT/rowspec_$sc.err; exit 2; }
  cat $OUT/rowspec_$sc.jsonl
done
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py C4 main=main cull_b4=sail_amd/lib/variants/libsail_hip_cull_b4.so > $OUT/cull_b4_C4.jsonl 2> $OUT/cull_b4_C4.err || { tail $OUT/cull_b4_C4.err; exit 3; }
cat $OUT/cull_b4_C4.jsonl
