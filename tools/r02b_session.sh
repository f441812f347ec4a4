#!/bin/bash
# Round-2 (second half) GPU session: parity suite on the current build, variant timings (C2-shaped C1, C3, C4;
# every variant's accumulator checked bit-identical to the first), phase profiles. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-s1}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 2; }
  tail -1 $OUT/pytest.log
fi
for s in ${SCENES:-C1 C3 C4}; do
  timeout -k 10 300 python -u tools/variant_bench.py $s >> $OUT/variants.log 2>&1 || { tail $OUT/variants.log; exit 3; }
done
cat $OUT/variants.log
if [ -d sail_amd/lib/phase ]; then
  for v in sail_amd/lib/phase/*.so; do
    timeout -k 10 300 python -u tools/phase_profile.py $v ${SCENES:-C1 C3 C4} > $OUT/phase_$(basename $v .so).log 2>&1 || { tail $OUT/phase_$(basename $v .so).log; exit 4; }
  done
  tail -n +1 $OUT/phase_*.log
fi
echo session ok
