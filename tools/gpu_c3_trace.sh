#!/bin/bash
# rocprofv3 kernel trace of N C3 scans (default 400) and the per-queue timeline of a few scans (tools/trace_lanes.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3t; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --workload c3 --steps ${N:-400} --warmup 5 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo "c3 trace failed"; tail -3 $O/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); print('c3', d['value'], d['steps'], d.get('breakdown_ms_per_step'))"
python3 tools/trace_lanes.py $O/prof/run_kernel_trace.csv 200 6 > $O/lanes.txt; tail -60 $O/lanes.txt
python3 tools/ktimed.py $O/prof/run_kernel_trace.csv 5 ${N:-400} > $O/c3_timed.txt; head -25 $O/c3_timed.txt
