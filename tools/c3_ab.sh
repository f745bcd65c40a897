#!/bin/bash
# Bench A/B of one workload (WL, default the C3 replay; STEPS) for each library given (product or `make VARIANT=`
# builds), R rounds interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WL=${WL:-c3}; STEPS=${STEPS:-1500}; R=${R:-2}
for r in $(seq 1 $R); do
  for lib in "$@"; do
    o=gpurun_out/ab_${WL}_$lib.$r
    NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload $WL --steps $STEPS --warmup 5 --no-cpu-baseline > $o.json 2> $o.err || { echo "$lib failed"; tail -3 $o.err; exit 1; }
    python3 -c "import json; d=json.load(open('$o.json')); print('$WL $lib', d['value'], d.get('breakdown_ms_per_step'))"
  done
done
