#!/bin/bash
# k_fitness workgroup cap A/B (NDT_FIT_WG) on the C3 replay: rocprofv3 kernel statistics per value.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for wg in "$@"; do
  d=gpurun_out/fwg_$wg; rm -rf $d
  NDT_FIT_WG=$wg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload c3 --steps 300 --warmup 5 --no-cpu-baseline > $d.json 2> $d.err || { echo "wg=$wg failed"; tail -3 $d.err; exit 1; }
  echo "== wg=$wg $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))")"
  python3 tools/kstats.py $d/run_kernel_stats.csv 305 > $d.txt; grep -E "fitness" $d.txt
done
