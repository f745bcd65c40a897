#!/bin/bash
# GPU tests, then a rocprofv3 kernel trace of a short default bench (kernel table + bench line).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t.out 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/t.out
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/pv
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pv -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pv.json 2> gpurun_out/pv.err || exit 1
python3 tools/kstats.py gpurun_out/pv/run_kernel_stats.csv 13 | head -14
python3 -c "import json; d=json.loads(open('gpurun_out/pv.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))"
