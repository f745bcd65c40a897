set -o pipefail
mkdir -p gpurun_out/c4q
for cfg in "4 3" "8 3" "8 4" "8 6" "16 8"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 NDT_BATCH_STREAMS=$2 timeout -k 10 300 python bench.py --workload c4 --steps 1024 --no-cpu-baseline > gpurun_out/c4q/c4_q$1_s$2.json 2> gpurun_out/c4q/c4_q$1_s$2.err || { echo "c4 q$1 s$2 failed"; tail -3 gpurun_out/c4q/c4_q$1_s$2.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4q/c4_q$1_s$2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('q$1 s$2', d['value'], r.get('ms_per_launch'), r.get('frac'), r.get('aggregate_frac'))"
done
