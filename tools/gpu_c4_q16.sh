#!/bin/bash
# C4 with more registrations in flight than hardware queues allow in dispatch order: 16 queues x 8 streams (the round-5
# configuration whose radix look-back timed out), and the default 4 x 3, 1024 pairs each; reports the target builds
# re-run after a flagged sort.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4q; mkdir -p $O
# CFGS: comma-separated "queues streams" pairs
IFS=, read -ra LIST <<< "${CFGS:-16 8,4 3}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 NDT_BATCH_STREAMS=$2 timeout -k 10 300 python bench.py --workload c4 --steps 1024 --no-cpu-baseline > $O/c4_q$1_s$2.json 2> $O/c4_q$1_s$2.err || { echo "c4 q$1 s$2 failed"; tail -3 $O/c4_q$1_s$2.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_q$1_s$2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('q$1 s$2', d['value'], r.get('ms_per_launch'), r.get('aggregate_frac'), d.get('target_builds'), d['config']['converged'])"
done
