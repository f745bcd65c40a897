#!/bin/bash
# C3 CU-partition A/B (NDT_LANE_CUS side-lane CUs, NDT_LANE_CU_MODE): 2000-scan replays, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3cus; mkdir -p $O
for rep in 1 2; do
  for cfg in ${CFGS:-0:0 32:0 64:0 32:1 64:1}; do
    k=${cfg%:*}; m=${cfg#*:}
    f=$O/c3_${rep}_${k}_${m}.json
    if [ "$k" = "0" ]; then env -u NDT_LANE_CUS timeout -k 10 300 python bench.py --workload c3 --steps ${STEPS:-2000} --warmup 5 --no-cpu-baseline > $f 2> $f.err || { echo "c3 $cfg failed"; tail -3 $f.err; exit 1; }
    else NDT_LANE_CUS=$k NDT_LANE_CU_MODE=$m timeout -k 10 300 python bench.py --workload c3 --steps ${STEPS:-2000} --warmup 5 --no-cpu-baseline > $f 2> $f.err || { echo "c3 $cfg failed"; tail -3 $f.err; exit 1; }; fi
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('c3 $rep cus=$k mode=$m', d['value'], d['breakdown_ms_per_step'])"
  done
done
echo done
