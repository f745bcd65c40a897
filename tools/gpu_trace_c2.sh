#!/bin/bash
# rocprofv3 kernel trace of a short default (C2) bench and of C5, kept for tools/step_timeline.py / tools/ktimed.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/trace; rm -rf $O; mkdir -p $O
for wl in ${WLS:-c2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$wl -o run --output-format csv -- python3 bench.py --workload $wl --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { echo "$wl failed"; tail -5 $O/$wl.err; exit 1; }
  python3 tools/step_timeline.py $O/$wl/run_kernel_trace.csv > $O/${wl}_timeline.txt
  python3 tools/ktimed.py $O/$wl/run_kernel_trace.csv 3 ${STEPS:-10} > $O/${wl}_timed.txt
  echo "== $wl $(python3 -c "import json; d=json.loads(open('$O/$wl.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  cat $O/${wl}_timeline.txt
done
