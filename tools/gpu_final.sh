#!/bin/bash
# All GPU tests + smoke + short C2 line (gpu_tests.sh), then the C3 replay line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
timeout -k 10 600 python bench.py --workload c3 --steps 1500 --warmup 5 > gpurun_out/c3.json 2> gpurun_out/c3.err || { echo "c3 failed"; tail -5 gpurun_out/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/c3.json').read().strip().splitlines()[-1]); print('c3', d['value'], d.get('breakdown_ms_per_step'))"
