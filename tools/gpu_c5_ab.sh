#!/bin/bash
# C5 pass geometry A/B (NDT_PPT: 2 = two points per thread with a tile loop, 3 = grid of one-tile workgroups with the
# two-level hand-off): the C5 full-size parity tests under each, then single-pass micro timings and bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c5ab; mkdir -p $O
for ppt in ${PPTS:-3}; do
  NDT_PPT=$ppt timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_config.py -k c5 -m gpu -x -v -s --timeout 500 --timeout-method thread > $O/pytest_$ppt.log 2>&1; rc=$?
  echo "ppt $ppt pytest rc=$rc"; grep -E "PASSED|FAILED|C5:" $O/pytest_$ppt.log | tail -3
  [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest_$ppt.log | head; exit $rc; }
done
for rep in 1 2; do
  for ppt in ${BENCH_PPTS:-2 3}; do
    f=$O/c5_${rep}_$ppt.json
    NDT_PPT=$ppt timeout -k 10 300 python bench.py --workload c5 --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $f 2> $f.err || { echo "c5 $ppt failed"; tail -3 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('c5 $rep ppt$ppt', d['value'], r.get('ms_per_launch'), r.get('frac'))"
  done
done
echo done
