#!/bin/bash
# Kernel-time A/B: one rocprofv3 kernel trace per ';'-separated "ENV=VAL ..." variant of one workload; prints the
# per-kernel averages of the kernels matching KPAT.  WL, STEPS, KPAT, VARS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${WL:-c3}; STEPS=${STEPS:-100}; KPAT=${KPAT:-k_fitness}
IFS=';' read -ra VL <<< "${VARS:-}"
n=0
for v in "${VL[@]}"; do
  n=$((n+1)); d=gpurun_out/kv_$n; rm -rf $d
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 2 --no-cpu-baseline > $d.json 2> $d.err || { echo "variant '$v' failed"; tail -3 $d.err; exit 1; }
  echo "== $v : $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))")"
  python3 tools/kstats.py $d/run_kernel_stats.csv $STEPS | grep -E "$KPAT"
done
