#!/bin/bash
# C3 at its configuration: the whole 4541-scan replay with its CPU baseline, then a rocprofv3 kernel-trace of the
# first 1000 scans (kernel statistics per scan).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u bench.py --workload c3 --save-traj $O/c3_traj.npz > $O/c3_4541.json 2> $O/c3_4541.err || { echo "c3 failed"; tail -5 $O/c3_4541.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3_4541.json').read().strip().splitlines()[-1]); print('c3', d['value'], d['steps'], d['breakdown_ms_per_step'], d['roofline']['ms_per_launch'], d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload c3 --steps 1000 --warmup 5 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || { echo "rocprof failed"; tail -3 $O/prof.err; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 1000 > $O/rocprof_c3_summary.txt; head -16 $O/rocprof_c3_summary.txt
rm -f $O/prof/run_kernel_trace.csv
echo c3 session done
