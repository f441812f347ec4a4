set -o pipefail
O=gpurun_out/s3; mkdir -p $O
V="base=main:9=0 pool=main:9=1 poolG1=main:9=1,4=1 poolG2=main:9=1,4=2 poolG16=main:9=1,4=16 m64=sail_amd/lib/variants/libsail_hip_m64.so:9=1 m128=sail_amd/lib/variants/libsail_hip_m128.so:9=1 m256=sail_amd/lib/variants/libsail_hip_m256.so:9=1"
VARIANT_ROUNDS=1 timeout -k 10 400 python -u tools/variant_bench.py C1 $V > $O/var_c1.jsonl 2>&1 || { tail $O/var_c1.jsonl; exit 2; }
cat $O/var_c1.jsonl | cut -c1-160
VARIANT_ROUNDS=1 timeout -k 10 400 python -u tools/variant_bench.py C3 $V rp448=sail_amd/lib/variants/libsail_hip_rp448.so:9=1 > $O/var_c3.jsonl 2>&1 || { tail $O/var_c3.jsonl; exit 3; }
cat $O/var_c3.jsonl | cut -c1-160
PHASE_DEBUG=9=1 timeout -k 10 300 python -u tools/phase_profile.py sail_amd/lib/libsail_hip_phase.so C1 C3 > $O/phases_pool.jsonl 2>&1 || exit 4
cat $O/phases_pool.jsonl
PMC_OUT=$O/pmc_c2_pool PMC_CONFIG=C2 PMC_SPP=64 PMC_BENCH_ARGS="--debug 9=1" bash tools/pmc.sh > /dev/null || exit 5
python tools/pmc_summary.py $O/pmc_c2_pool $O/pmc_c2_pool.json 2073600 32 8 cornell_box_readme_C2 | grep -A12 derived
PMC_OUT=$O/pmc_c3_pool PMC_CONFIG=C3 PMC_SPP=64 PMC_BENCH_ARGS="--debug 9=1" bash tools/pmc.sh > /dev/null || exit 6
python tools/pmc_summary.py $O/pmc_c3_pool $O/pmc_c3_pool.json 2073600 32 8 materials_demo_C3 | grep -A12 derived
