#!/bin/bash
# Round 6 check: the new / touched GPU tests on the default library, then C2 bench lines of LIBS interleaved (A/B).
#   LIBS="libndt_hip.so libndt_hip_tf1.so" TESTS="tests/test_x.py ..." bash tools/gpu_r6_check.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|C2 pair|C5:" $O/pytest.log | tail -40
  [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit $rc; }
fi
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-libndt_hip.so}; do
    for wl in ${BENCH:-c2}; do
      f=$O/${wl}_${rep}_$lib.json
      NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline ${BENCH_ARGS} > $f 2> $f.err || { echo "$wl $lib failed"; tail -3 $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl $rep $lib', d['value'], r.get('ms_per_launch'), r.get('frac'), r.get('aggregate_frac'))"
    done
  done
done
echo done
