#!/bin/bash
# Leading-tail chain (NDT_LEAD_TAIL=1, default) against the last-workgroup tails (0) on C2, C5, C3 and C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # label, env, bench args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu-baseline > gpurun_out/la.json 2> gpurun_out/la.err || { echo "$1 failed"; tail -3 gpurun_out/la.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/la.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$1', d['value'], d.get('breakdown_ms_per_step'), r.get('ms_per_launch'), r.get('frac'))"
}
for v in 1 0; do
  run "c2 lead=$v" "NDT_LEAD_TAIL=$v" "--steps 300 --warmup 5"
  run "c5 lead=$v" "NDT_LEAD_TAIL=$v" "--workload c5 --steps 20 --warmup 2"
  run "c3 lead=$v" "NDT_LEAD_TAIL=$v" "--workload c3 --steps 600 --warmup 5"
  run "c4 lead=$v" "NDT_LEAD_TAIL=$v" "--workload c4 --steps 256 --warmup 4"
done
