#!/bin/sh
# Builds the CPU parity oracle (test infrastructure). Outputs only under oracle/build/.
set -e
cd "$(dirname "$0")"
mkdir -p build
CXX=${CXX:-g++}
FLAGS="-O2 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -Wall -Wextra -Wno-unused-function"
$CXX $FLAGS sail_oracle.cpp -o build/libsail_oracle.so
$CXX $FLAGS -DSAIL_COUNT_OPS sail_oracle.cpp -o build/libsail_oracle_count.so
