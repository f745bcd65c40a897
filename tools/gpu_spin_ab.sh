#!/bin/bash
# C2 / C4 bench lines with the align's host wait spinning on the read-back word (NDT_SPIN_WAIT=1, default) and with a
# stream synchronisation (0), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sp in 1 0 1 0; do
  NDT_SPIN_WAIT=$sp timeout -k 10 240 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > gpurun_out/spin_$sp.json 2> gpurun_out/spin_$sp.err || { echo "bench $sp failed"; tail -3 gpurun_out/spin_$sp.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/spin_$sp.json')); print('c2 spin=$sp', d['value'], d['ms_per_step'], d['breakdown_ms_per_step'])"
done
for sp in 1 0; do
  NDT_SPIN_WAIT=$sp timeout -k 10 300 python3 bench.py --workload c4 --steps 256 --warmup 8 --no-cpu-baseline > gpurun_out/spin4_$sp.json 2> gpurun_out/spin4_$sp.err || { echo "c4 $sp failed"; tail -3 gpurun_out/spin4_$sp.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/spin4_$sp.json')); print('c4 spin=$sp', d['value'])"
done
