#!/bin/bash
# A/B of variant libraries on one box: parity subset of each variant (TESTLIBS), single-pass kernel time of each library
# (tools/pass_micro.py under rocprofv3; MICRO "wl:ppt" list), then the C2 and C4 bench lines of each library, interleaved
# twice.   LIBS="libndt_hip.so libndt_hip_x.so" TESTLIBS="libndt_hip_x.so" bash tools/gpu_libs_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/libs; rm -rf $O; mkdir -p $O
LIBS=${LIBS:-libndt_hip.so}
if [ -n "$PRODTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_prod.log 2>&1; rc=$?
  echo "product pytest rc=$rc"; grep -E "passed|failed" $O/pytest_prod.log | tail -2
  [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest_prod.log | head -20; exit $rc; }
fi
for lib in $TESTLIBS; do
  NDT_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lead.py tests/test_gpu_fullsize.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_$lib.log 2>&1; rc=$?
  echo "$lib pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_$lib.log | tail -8
  [ $rc -gt 1 ] && exit $rc
done
for v in ${MICRO:-c5:2 c2:1}; do
  wl=${v%:*}; ppt=${v#*:}
  for lib in $LIBS; do
    d=$O/${wl}_p${ppt}_$lib
    MICRO_PPT=$ppt NDT_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/pass_micro.py $wl 20 > $d.out 2> $d.err || { echo "$lib $wl failed"; tail -3 $d.err; exit 1; }
    echo "== $wl ppt$ppt $lib $(tail -1 $d.out | cut -c1-110)"
    python3 tools/kstats.py $d/run_kernel_stats.csv 1 | grep -E "k_pass"
    rm -f $d/run_kernel_trace.csv
  done
done
for rep in 1 2; do
  for lib in $LIBS; do
    for wl in ${BENCH:-c2 c4}; do
      f=$O/${wl}_${rep}_$lib.json
      NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > $f 2> $f.err || { echo "$wl $lib failed"; tail -3 $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl $rep $lib', d['value'], r.get('ms_per_launch'), r.get('frac'), r.get('aggregate_frac'))"
    done
  done
done
echo done
