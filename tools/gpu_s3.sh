#!/bin/bash
# Session A/B at one box: GPU tests at the default build, then C5 / C2 bench lines per variant library (LIBS), then the
# C4 line per variant (C4_LIBS).  Every step under its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/s3; rm -rf $O; mkdir -p $O
if [ -n "${TESTS-x}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -12
  [ $rc -gt 1 ] && exit $rc
fi
for lib in ${LIBS:-libndt_hip.so}; do
  for wl in ${WLS:-c5 c2}; do
    st=100; [ $wl = c5 ] && st=10
    NDT_HIP_LIB=$lib timeout -k 10 400 python bench.py --workload $wl --steps $st --warmup 2 --no-cpu-baseline > $O/${wl}_$lib.json 2> $O/${wl}_$lib.err || { echo "$wl $lib failed"; tail -5 $O/${wl}_$lib.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${wl}_$lib.json')); r=d['roofline']; print('$wl', '$lib', d['value'], r.get('ms_per_launch'), r.get('frac'))"
  done
done
for lib in ${C4_LIBS-}; do
  NDT_HIP_LIB=$lib timeout -k 10 400 python bench.py --workload c4 --steps ${C4_STEPS:-512} --warmup 8 --no-cpu-baseline > $O/c4_$lib.json 2> $O/c4_$lib.err || { echo "c4 $lib failed"; tail -5 $O/c4_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$lib.json')); r=d['roofline']; print('c4', '$lib', d['value'], r.get('ms_per_launch'), r.get('frac'), r.get('aggregate_frac'))"
done
echo s3 done
