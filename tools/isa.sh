#!/bin/sh
# Disassembles the gfx950 code object of sail_trace.hip (extra hipcc flags in "$@") with source-line tables:
# writes /tmp/isa/trace_g.s, one block per kernel. tools/isa_attr.py then attributes instructions to source lines.
set -e
cd "$(dirname "$0")/../sail_amd"
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wno-unused-function \
  --offload-arch=gfx950 --cuda-device-only -gline-tables-only "$@" -c csrc/sail_trace.hip -o /tmp/isa/trace_dev_g.o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/isa/trace_dev_g.o \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/isa/trace_g.co
/opt/rocm/lib/llvm/bin/llvm-objdump -d -l --no-show-raw-insn /tmp/isa/trace_g.co > /tmp/isa/trace_g.s
