#!/bin/sh
# Per-kernel VGPRs / occupancy / spills of sail_trace.hip (or $1 with extra flags $2...) from the compiler's
# resource-usage remarks.
cd "$(dirname "$0")/../sail_amd"
src=${1:-csrc/sail_trace.hip}; [ $# -gt 0 ] && shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-function --offload-arch=gfx950 \
  -Icsrc "$@" -c "$src" -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|SGPRs Spill|VGPRs Spill|Occupancy" | sed 's/.*remark: //; s/ \[-Rpass.*//' |
  paste -d' ' - - - - - | sed 's/Function Name: //; s/Occupancy \[waves\/SIMD\]/waves/'
rm -f /tmp/regs_$$.o
