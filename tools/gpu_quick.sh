#!/bin/bash
# Quick bench lines: C2 (300 steps, twice) and C5 (20 steps), no CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > gpurun_out/q_c2_$i.json 2> gpurun_out/q_c2_$i.err || { echo "c2 failed"; tail -3 gpurun_out/q_c2_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/q_c2_$i.json')); print('c2', d['value'], d['ms_per_step'], d['breakdown_ms_per_step'], d['roofline'].get('phases_ms'))"
done
timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/q_c5.json 2> gpurun_out/q_c5.err || { echo "c5 failed"; tail -3 gpurun_out/q_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/q_c5.json')); print('c5', d['value'], d['ms_per_step'], d['breakdown_ms_per_step'], d['roofline'].get('phases_ms'))"
