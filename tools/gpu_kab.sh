#!/bin/bash
# rocprofv3 kernel statistics of one workload for the product library and one variant library (VAR=name).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${WL:-c5}; STEPS=${STEPS:-5}; VAR=${VAR:-nt}
for lib in libndt_hip.so libndt_hip_$VAR.so; do
  d=gpurun_out/kab_$lib; rm -rf $d
  NDT_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 2 --no-cpu-baseline > $d.json 2> $d.err || { echo "$lib failed"; tail -3 $d.err; exit 1; }
  echo "== $lib $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))")"
  python3 tools/kstats.py $d/run_kernel_stats.csv $((STEPS+2)) | head -12
done
