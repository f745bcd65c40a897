#!/bin/bash
# All GPU tests + smoke + short C2 line, then the front-end line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --workload fe --steps 200 --warmup 3 > gpurun_out/fe.json 2> gpurun_out/fe.err || { echo "fe failed"; tail -5 gpurun_out/fe.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/fe.json').read().strip().splitlines()[-1]); print('fe', d['value'])"
