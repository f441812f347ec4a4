#!/bin/bash
# Variant timings (sail_amd/lib/variants/*.so, built by tools/build_variants.sh): C2-shaped C1, C3, C4; every
# variant's accumulator must be bit-identical to the first. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03_var}
mkdir -p $OUT
for s in ${SCENES:-C1 C3 C4}; do
  timeout -k 10 400 python -u tools/variant_bench.py $s >> $OUT/variants.log 2>&1 || { tail $OUT/variants.log; exit 3; }
done
cat $OUT/variants.log | cut -c1-200
echo variants ok
