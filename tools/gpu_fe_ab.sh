#!/bin/bash
# Front-end A/B: front-end GPU tests with each library, then the fe workload under rocprofv3 (k_sor_knn line).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  d=gpurun_out/feab_$lib; rm -rf $d
  NDT_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_front_end.py -m gpu -x -q --timeout 120 --timeout-method thread > $d.tests.log 2>&1 || { echo "$lib fe tests failed"; tail -20 $d.tests.log; exit 1; }
  echo "$lib $(tail -1 $d.tests.log)"
  NDT_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload fe --steps 100 --warmup 3 --no-cpu-baseline > $d.json 2> $d.err || { echo "$lib failed"; tail -3 $d.err; exit 1; }
  echo "== $lib $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'])")"
  python3 tools/kstats.py $d/run_kernel_stats.csv 103 > $d.txt; grep -E "sor_knn|total" $d.txt
done
