set -o pipefail
O=gpurun_out/s7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "jit or room or phase" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_jit.log 2>&1; rc=$?; tail -3 $O/pytest_jit.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_jit.log | head; exit 2; }
for sc in ALL AREA BILERP AREA0; do
  VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py $sc jit=main:9=1 jitroom=main:9=9 > $O/var_fam_$sc.jsonl 2>&1 || { tail $O/var_fam_$sc.jsonl; exit 3; }
  cut -c1-150 $O/var_fam_$sc.jsonl
done
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py C3 base=main old=sail_amd/lib/variants/libsail_hip_r4base.so jit=main:9=5 > $O/var_c3.jsonl 2>&1 || { tail $O/var_c3.jsonl; exit 4; }
cut -c1-150 $O/var_c3.jsonl
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py UI base=main jit=main:9=5 > $O/var_ui.jsonl 2>&1 || { tail $O/var_ui.jsonl; exit 5; }
cut -c1-150 $O/var_ui.jsonl
VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py C4 base=main jit=main:9=3 > $O/var_c4.jsonl 2>&1 || { tail $O/var_c4.jsonl; exit 6; }
cut -c1-150 $O/var_c4.jsonl
for sc in C1 C3 C4; do
  VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py $sc base=main w2l_rcp2=sail_amd/lib/variants/libsail_hip_w2l_rcp2.so > $O/var_w2l_$sc.jsonl 2>&1 || { tail $O/var_w2l_$sc.jsonl; exit 8; }
  cut -c1-150 $O/var_w2l_$sc.jsonl
done
