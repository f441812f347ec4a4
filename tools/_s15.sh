set -o pipefail
O=gpurun_out/s15; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_jit_fallback.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_fallback.log 2>&1; rc=$?; tail -3 $O/pytest_fallback.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest_fallback.log | head; exit 2; }
for sc in C1 C3; do
  VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py $sc r36=main r18=main:7=18 r72=main:7=72 > $O/var_rounds_$sc.jsonl 2>&1 || { tail $O/var_rounds_$sc.jsonl; exit 3; }
  cut -c1-150 $O/var_rounds_$sc.jsonl
done
VARIANT_ROUNDS=2 timeout -k 10 500 python -u tools/variant_bench.py C4 r64=main r32=main:8=32 r128=main:8=128 > $O/var_rounds_C4.jsonl 2>&1 || { tail $O/var_rounds_C4.jsonl; exit 4; }
cut -c1-150 $O/var_rounds_C4.jsonl
