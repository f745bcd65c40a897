#!/bin/bash
# k_fitness kernel time per library over a short C3 replay (rocprofv3 --kernel-trace --stats):  bash tools/gpu_fit_kstats.sh libA.so libB.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fitk; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    d=$O/${rep}_$lib
    NDT_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload c3 --steps 400 --warmup 5 --no-cpu-baseline > $d.json 2> $d.err || { echo "$lib failed"; tail -3 $d.err; exit 1; }
    echo "== $rep $lib $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'])")"
    python3 tools/kstats.py $d/run_kernel_stats.csv 1 | grep -E "k_fitness|k_fit_tables|k_pass_lead"
    rm -f $d/run_kernel_trace.csv
  done
done
