#!/bin/bash
# Round-3 study call: per-rank scaling emulation (C4 with the host's sample-group rule and with groups forced
# 1/2/4, C3, C5 sample split) and the dynamic VALU instruction mix of the C3 room kernel and the C2 Cornell kernel.
# Each GPU step has its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION_OUT:-r03_study}
mkdir -p $OUT
P="timeout -k 10 300 python -u tools/scaling_probe.py"
$P C4 32 > $OUT/scale_c4_auto.jsonl 2>&1 || { tail $OUT/scale_c4_auto.jsonl; exit 2; }
for g in 1 2 4; do $P C4 32 --groups $g > $OUT/scale_c4_g$g.jsonl 2>&1 || { tail $OUT/scale_c4_g$g.jsonl; exit 3; }; done
for g in 2 4; do $P C4 32 --groups $g --lib sail_amd/lib/variants/libsail_hip_g_cullg1024.so > $OUT/scale_c4_g${g}_nt1024.jsonl 2>&1 || { tail $OUT/scale_c4_g${g}_nt1024.jsonl; exit 3; }; done
$P C3 256 > $OUT/scale_c3.jsonl 2>&1 || { tail $OUT/scale_c3.jsonl; exit 4; }
$P C5 256 > $OUT/scale_c5.jsonl 2>&1 || { tail $OUT/scale_c5.jsonl; exit 5; }
$P C2 256 > $OUT/scale_c2.jsonl 2>&1 || { tail $OUT/scale_c2.jsonl; exit 6; }
cat $OUT/scale_*.jsonl | cut -c1-220
PMC_OUT=$OUT/mix_c3 PMC_CONFIG=C3 PMC_SPP=64 bash tools/pmc_mix.sh > /dev/null || exit 7
PMC_OUT=$OUT/mix_c2 PMC_CONFIG=C2 PMC_SPP=64 bash tools/pmc_mix.sh > /dev/null || exit 8
python tools/pmc_mix_summary.py $OUT/mix_c3 $OUT/r03_pmc_valu_mix_c3.json 2073600 32 8 materials_demo_C3 889.32 || exit 9
python tools/pmc_mix_summary.py $OUT/mix_c2 $OUT/r03_pmc_valu_mix_c2.json 2073600 32 8 cornell_box_readme_C2 298.98 || exit 9
echo study ok
