#!/bin/bash
# Full GPU session: all gpu tests, smoke, the default bench line (C2 + CPU baseline), a rocprofv3 kernel-trace of a
# short C2 bench, then the other workloads (C5 dense stress, front end, C3 replay, C4 batched).  Every step has its own time limit;
# the session stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
rm -rf $O/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof failed"; exit 1; }
timeout -k 10 400 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; exit 1; }
timeout -k 10 300 python bench.py --workload fe --steps 40 --warmup 3 > $O/fe.json 2> $O/fe.err || { echo "fe failed"; exit 1; }
timeout -k 10 600 python bench.py --workload c3 --steps 1500 --warmup 5 > $O/c3.json 2> $O/c3.err || { echo "c3 failed"; exit 1; }
timeout -k 10 400 python bench.py --workload c4 --steps 512 --warmup 4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; exit 1; }
rm -rf $O/prof5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_c5.json 2> $O/prof_c5.err || { echo "rocprof c5 failed"; exit 1; }
echo session done
