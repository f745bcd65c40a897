#!/bin/bash
# getFitnessScore check + A/B: the fitness / odom GPU tests, then the C3 replay with the product library and with the
# libraries named as arguments (rocprofv3 kernel statistics, k_fitness line), one run each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fitness or odom" > gpurun_out/fit_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fit_tests.log; exit 1; }
tail -1 gpurun_out/fit_tests.log
for lib in libndt_hip.so "$@"; do
  d=gpurun_out/fab_$lib; rm -rf $d
  NDT_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fitness" > $d.tests.log 2>&1 || { echo "$lib fitness tests failed"; tail -30 $d.tests.log; exit 1; }
  echo "$lib $(tail -1 $d.tests.log)"
  NDT_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload c3 --steps 300 --warmup 5 --no-cpu-baseline > $d.json 2> $d.err || { echo "$lib failed"; tail -3 $d.err; exit 1; }
  echo "== $lib $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))")"
  python3 tools/kstats.py $d/run_kernel_stats.csv 305 > $d.txt; grep -E "fitness|total" $d.txt
done
