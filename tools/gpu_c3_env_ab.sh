#!/bin/bash
# C3 A/B of an environment switch (VAR, default NDT_ODOM_FIT_LATE): unset vs =1, interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VAR=${VAR:-NDT_ODOM_FIT_LATE}
O=gpurun_out/c3env; rm -rf $O; mkdir -p $O
for rep in 1 2 3; do
  for v in off on; do
    f=$O/c3_${rep}_$v.json
    if [ $v = on ]; then export $VAR=1; else unset $VAR; fi
    timeout -k 10 300 python bench.py --workload c3 --steps ${STEPS:-2000} --warmup 5 --no-cpu-baseline > $f 2> $f.err || { echo "c3 $v failed"; tail -3 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('c3 $rep $VAR=$v', d['value'], d['roofline'].get('ms_per_launch'), d['breakdown_ms_per_step'])"
  done
done
unset $VAR
echo done
