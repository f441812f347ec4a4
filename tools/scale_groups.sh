#!/bin/bash
# Per-rank throughput (tools/scaling_probe.py, world sizes emulated on one GPU) against the sample-group count and, for
# the Cornell form, the samples in flight per workgroup: the data behind the host's rules for the run-time kernels
# (sail_capi.cpp jitNsFor and the group rule; profiles/r05_scale_groups_c2.jsonl, _c4.jsonl, r05_scale_ns_c2.jsonl).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05f; mkdir -p $O
for g in 1 2 4; do timeout -k 10 300 python -u tools/scaling_probe.py C2 1024 --groups $g --worlds 1,4,8 --debug 11=16 >> $O/scale_groups_c2.jsonl 2>&1 || exit 3; done
for g in 1 2 4 8; do timeout -k 10 300 python -u tools/scaling_probe.py C4 32 --groups $g --worlds 1,2,4,8 >> $O/scale_groups_c4.jsonl 2>&1 || exit 4; done
for ns in 1 4 16; do for g in 0 1; do
  a=""; [ $g -gt 0 ] && a="--groups $g"
  timeout -k 10 300 python -u tools/scaling_probe.py C2 1024 $a --worlds 1,4,8 --debug 11=$ns >> $O/scale_ns_c2.jsonl 2>&1 || exit 5
done; done
echo ok
