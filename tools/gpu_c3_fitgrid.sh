#!/bin/bash
# C3 with getFitnessScore's grid capped (NDT_FIT_GRID workgroups of NDT_FIT_BLOCK threads, grid-stride over the
# queries), interleaved on one box:   GRIDS="0 2048 512" bash tools/gpu_c3_fitgrid.sh   (0 = the library default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3grid; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for g in ${GRIDS:-0 2048 512}; do
    f=$O/c3_${rep}_$g.json
    if [ "$g" = 0 ]; then unset NDT_FIT_GRID; else export NDT_FIT_GRID=$g; fi
    timeout -k 10 300 python bench.py --workload c3 --steps ${STEPS:-2000} --warmup 5 --no-cpu-baseline > $f 2> $f.err || { echo "c3 grid $g failed"; tail -3 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('c3 $rep grid $g', d['value'], d['roofline'].get('ms_per_launch'))"
  done
done
unset NDT_FIT_GRID
echo done
