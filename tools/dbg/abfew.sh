set -u
for v in 4096 1024 512 256 128; do
  DQ_FREQ_FEW_BLOCKS=$v timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/abfew_$v.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/abfew_$v.log') if l.startswith('{')][-1]);print($v, round(d['ms_per_step'],2))"
done
