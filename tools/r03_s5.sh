#!/bin/bash
# Occupancy / barrier / priority variants of the adopted kernels (C1, C3, C4), then the C2 PMC passes of the
# adopted build (profiles/r03_pmc_summary.json). Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03i}
mkdir -p $OUT
SESSION_OUT=${SESSION_OUT:-r03i} SCENES="C1 C3 C4" bash tools/r03_variants.sh || exit 2
PMC_OUT=$OUT/pmc_c2 bash tools/pmc.sh || exit 3
echo s5 ok
