#!/bin/bash
# rocprofv3 kernel statistics + bench value of one workload (WL, STEPS) under each environment setting given as an
# argument (e.g. NDT_SORTED_FINALIZE_MIN=0), for A/B runs of runtime switches without a rebuild.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${WL:-c5}; STEPS=${STEPS:-5}
i=0
for spec in "$@"; do
  i=$((i+1)); d=gpurun_out/envab_${WL}_$i; rm -rf $d
  env $spec true || exit 1
  export $spec
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 2 --no-cpu-baseline > $d.json 2> $d.err || { echo "$spec failed"; tail -3 $d.err; exit 1; }
  unset ${spec%%=*}
  echo "== $spec $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))")"
  python3 tools/kstats.py $d/run_kernel_stats.csv $((STEPS+2)) > $d.txt; head -14 $d.txt
done
