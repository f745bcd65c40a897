#!/bin/bash
# Profiling-build phase breakdown (in-kernel stamps) of the C2 bench for each library in LIBS (interleaved REPS times).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/phases; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-libndt_hip_dbg.so}; do
    f=$O/${rep}_$lib.json
    NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload ${WL:-c2} --no-cpu-baseline ${BENCH_ARGS} > $f 2> $f.err || { echo "$lib failed"; tail -3 $f.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$rep $lib', d['value'], r.get('ms_per_launch'))
for k in ('phases_ms','workgroup_phases_ms','tail_phases_ms'):
    v = r.get(k) or d.get(k)
    if v: print('  ', k, {a: round(b*1000, 2) for a, b in v.items()})
"
  done
done
