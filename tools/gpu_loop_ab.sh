#!/bin/bash
# A/B of bench's timed loop: lean C-ABI calls (default) vs the Python wrapper per step (BENCH_API_LOOP=1), C2, twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for m in 0 1; do
    BENCH_API_LOOP=$m timeout -k 10 200 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > gpurun_out/lab_${m}_${i}.json 2> gpurun_out/lab_${m}_${i}.err || { echo "c2 api=$m failed"; tail -5 gpurun_out/lab_${m}_${i}.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/lab_${m}_${i}.json')); print('api_loop=$m', d['value'], d['ms_per_step'], d['breakdown_ms_per_step'])"
  done
done
