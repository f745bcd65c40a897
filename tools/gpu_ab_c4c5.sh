#!/bin/bash
# A/B of LIBS on C4 (1024 pairs) and C5 (10 steps), interleaved REPS times, after TESTS on the default library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab45; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-libndt_hip.so}; do
    f=$O/c4_${rep}_$lib.json
    NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload c4 --steps 1024 --no-cpu-baseline > $f 2> $f.err || { echo "c4 $lib failed"; tail -3 $f.err; exit 1; }
    g=$O/c5_${rep}_$lib.json
    NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $g 2> $g.err || { echo "c5 $lib failed"; tail -3 $g.err; exit 1; }
    python3 -c "
import json
a=json.loads(open('$f').read().strip().splitlines()[-1]); b=json.loads(open('$g').read().strip().splitlines()[-1])
print('$rep $lib c4', a['value'], a['roofline'].get('ms_per_launch'), a.get('mean_translation_error_m'), '| c5', b['value'], b['roofline'].get('ms_per_launch'))"
  done
done
