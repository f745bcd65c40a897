#!/bin/bash
# C4 at its configuration (4096 pairs, 1 GPU) with roofline + CPU baseline, its rocprofv3 kernel statistics (256 pairs)
# and the FETCH_SIZE / WRITE_SIZE passes of the pass kernel (64 pairs, three streams in flight).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4; rm -rf $O; mkdir -p $O
timeout -k 10 600 python bench.py --workload c4 > $O/c4_4096.json 2> $O/c4_4096.err || { echo "c4 failed"; tail -5 $O/c4_4096.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c4_4096.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['roofline'], d.get('cpu_baseline'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload c4 --steps 256 --warmup 8 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || { echo "rocprof failed"; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 256 > $O/rocprof_c4_summary.txt; head -12 $O/rocprof_c4_summary.txt
python3 tools/ktimed.py $O/prof/run_kernel_trace.csv 8 256 > $O/rocprof_c4_timed.txt; head -4 $O/rocprof_c4_timed.txt; rm -f $O/prof/run_kernel_trace.csv
for g in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $g --kernel-include-regex "k_pass_direct" -d $O/pmc_$g -o run --output-format csv -- python3 bench.py --workload c4 --steps 64 --warmup 4 --no-cpu-baseline > $O/pmc_$g.out 2> $O/pmc_$g.err || { echo "pmc $g failed"; tail -3 $O/pmc_$g.err; exit 1; }
done
echo c4 session done
