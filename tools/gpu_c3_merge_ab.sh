#!/bin/bash
# C3 with merge-extended keyframe targets (default) against fresh builds (NDT_NO_TARGET_MERGE=1), interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3merge; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for v in merge fresh; do
    f=$O/c3_${rep}_$v.json
    if [ $v = fresh ]; then export NDT_NO_TARGET_MERGE=1; else unset NDT_NO_TARGET_MERGE; fi
    timeout -k 10 300 python bench.py --workload c3 --steps ${STEPS:-2000} --warmup 5 --no-cpu-baseline > $f 2> $f.err || { echo "c3 $v failed"; tail -3 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('c3 $rep $v', d['value'], d['roofline'].get('ms_per_launch'), d['breakdown_ms_per_step'])"
  done
done
unset NDT_NO_TARGET_MERGE
echo done
