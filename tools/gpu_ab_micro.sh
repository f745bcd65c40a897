#!/bin/bash
# GPU tests (one process, no -x: every failure listed) then tools/pass_micro.py under rocprofv3 for each variant
# library given, on the workloads in WLS (default "c5 c2"): single-pass kernel time of each library on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
if [ -n "$TESTS" ]; then
  NDT_HIP_LIB=${TESTLIB:-libndt_hip.so} timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -15
  [ $rc -gt 1 ] && exit $rc
fi
for wl in ${WLS:-c5 c2}; do
  for lib in "$@"; do
    d=$O/${wl}_$lib
    NDT_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/pass_micro.py $wl ${REPS:-20} > $d.out 2> $d.err || { echo "$lib $wl failed"; tail -3 $d.err; exit 1; }
    echo "== $wl $lib $(tail -1 $d.out | cut -c1-160)"
    python3 tools/kstats.py $d/run_kernel_stats.csv 1 | grep -E "k_pass"
    rm -f $d/run_kernel_trace.csv
  done
done
echo done
