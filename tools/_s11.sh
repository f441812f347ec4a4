set -o pipefail
O=gpurun_out/s11; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "jit or phase or kernel_selection" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_jit.log 2>&1; rc=$?; tail -3 $O/pytest_jit.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_jit.log | head; exit 2; }
for sc in C1 C3 UI ALL AREA BILERP; do
  VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py $sc sets=main:9=11 rows=main:9=27 > $O/var_rows_$sc.jsonl 2>&1 || { tail $O/var_rows_$sc.jsonl; exit 3; }
  cut -c1-150 $O/var_rows_$sc.jsonl
done
for r in 1 2; do for l in 32 64; do
  timeout -k 10 300 python bench.py --config C4 --launch-spp $l --no-cpu-baseline --steps 1 --warmup 1 > $O/launch_C4_${l}_${r}.json 2> $O/launch.err || { tail $O/launch.err; exit 5; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $O/launch_C4_${l}_${r}.json C4 $l | tee -a $O/launch.txt
  timeout -k 10 300 python bench.py --config C5 --spp 4096 --launch-spp $l --no-cpu-baseline --steps 1 --warmup 1 > $O/launch_C5_${l}_${r}.json 2> $O/launch.err || { tail $O/launch.err; exit 5; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $O/launch_C5_${l}_${r}.json C5 $l | tee -a $O/launch.txt
done; done
