#!/bin/bash
# All GPU tests (one process), smoke, then a short C2 bench line without the CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest_gpu.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('c2',d['value'],r['ms_per_launch'],r.get('phases_ms'))"
