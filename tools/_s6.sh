set -o pipefail
O=gpurun_out/s6; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -4 $O/pytest_gpu.log; grep -E "FAIL|Error" $O/pytest_gpu.log | head -5; [ $rc -ne 0 ] && exit 2
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py ALL generic=main:9=0 jit=main:9=1 > $O/var_all.jsonl 2>&1 || { tail $O/var_all.jsonl; exit 3; }
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py AREA generic=main:9=0 jit=main:9=1 > $O/var_area.jsonl 2>&1 || { tail $O/var_area.jsonl; exit 4; }
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py BILERP generic=main:9=0 jit=main:9=1 > $O/var_bilerp.jsonl 2>&1 || { tail $O/var_bilerp.jsonl; exit 5; }
cut -c1-170 $O/var_all.jsonl $O/var_area.jsonl $O/var_bilerp.jsonl
VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py C4 base=main kset_c4=sail_amd/lib/variants/libsail_hip_kset_c4.so jit2=main:9=2 > $O/var_c4.jsonl 2>&1 || { tail $O/var_c4.jsonl; exit 6; }
cut -c1-170 $O/var_c4.jsonl
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py C3 base=main kset_c3=sail_amd/lib/variants/libsail_hip_kset_c3.so > $O/var_c3.jsonl 2>&1 || { tail $O/var_c3.jsonl; exit 7; }
cut -c1-170 $O/var_c3.jsonl
for sc in C1 C3 C4; do
  VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py $sc base=main w2l_rcp2=sail_amd/lib/variants/libsail_hip_w2l_rcp2.so > $O/var_w2l_$sc.jsonl 2>&1 || { tail $O/var_w2l_$sc.jsonl; exit 8; }
  cut -c1-170 $O/var_w2l_$sc.jsonl
done
