#!/bin/bash
# rocprofv3 kernel trace of one bench workload: WL (default c3), STEPS; kernel table per step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${WL:-c3}; STEPS=${STEPS:-200}
rm -rf gpurun_out/pw_$WL
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pw_$WL -o run --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 2 --no-cpu-baseline > gpurun_out/pw_$WL.json 2> gpurun_out/pw_$WL.err || exit 1
python3 tools/kstats.py gpurun_out/pw_$WL/run_kernel_stats.csv $STEPS | head -24
python3 -c "import json; d=json.loads(open('gpurun_out/pw_$WL.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))"
