#!/bin/bash
# variants first (the quick decision), then the study passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r03_variants.sh || exit $?
bash tools/r03_study.sh || exit $?
