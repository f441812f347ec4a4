set -o pipefail
O=gpurun_out/r05g; mkdir -p $O; rm -f $O/scale_c2.jsonl
timeout -k 10 300 python -u tools/scaling_probe.py C2 1024 >> $O/scale_c2.jsonl 2>&1 || exit 3
timeout -k 10 300 python -u tools/scaling_probe.py C5 1024 >> $O/scale_c2.jsonl 2>&1 || exit 3
echo ok
