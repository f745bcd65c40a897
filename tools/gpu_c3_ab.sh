#!/bin/bash
# C3 A/B of two libraries on one box (odom tests of the first, then three interleaved C3 replays of 2000 scans each).
#   bash tools/gpu_c3_ab.sh libA.so libB.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3ab; rm -rf $O; mkdir -p $O
NDT_HIP_LIB=$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_odom.py tests/test_gpu_c3_fullsize.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest.log | head; exit $rc; }
for rep in 1 2 3; do
  for lib in "$@"; do
    f=$O/c3_${rep}_$lib.json
    NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload c3 --steps 2000 --warmup 5 --no-cpu-baseline > $f 2> $f.err || { echo "c3 $lib failed"; tail -3 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('c3 $rep $lib', d['value'], d['roofline'].get('ms_per_launch'))"
  done
done
