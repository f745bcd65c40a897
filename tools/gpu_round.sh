#!/bin/bash
# Full GPU session at HEAD: all gpu tests, smoke, the default bench line (C2 + CPU baseline), a rocprofv3 kernel trace
# of a short C2 bench, the C5 dense stress line and its kernel statistics, the front end.  Every step has its own time
# limit; the session stops at the first failure.  (C3 / C4 at their configurations: tools/gpu_c3.sh, tools/gpu_c4.sh;
# counter passes: tools/pmc.sh.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/round; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('c2', d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/prof_c2.json 2> $O/prof_c2.err || { echo "rocprof c2 failed"; exit 1; }
python3 tools/kstats.py $O/prof_c2/run_kernel_stats.csv 33 > $O/rocprof_c2_summary.txt
python3 tools/ktimed.py $O/prof_c2/run_kernel_trace.csv 3 30 > $O/rocprof_c2_timed.txt; rm -f $O/prof_c2/run_kernel_trace.csv
timeout -k 10 600 python bench.py --workload c5 --steps 20 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_c5.json 2> $O/prof_c5.err || { echo "rocprof c5 failed"; exit 1; }
python3 tools/kstats.py $O/prof_c5/run_kernel_stats.csv 7 > $O/rocprof_c5_summary.txt
python3 tools/ktimed.py $O/prof_c5/run_kernel_trace.csv 2 5 > $O/rocprof_c5_timed.txt; rm -f $O/prof_c5/run_kernel_trace.csv
timeout -k 10 300 python bench.py --workload fe --steps 200 --warmup 5 > $O/fe.json 2> $O/fe.err || { echo "fe failed"; exit 1; }
python3 -c "import json; d=json.load(open('$O/fe.json')); print('fe', d['value'])"
echo session done
