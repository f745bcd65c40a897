#!/bin/bash
# C2 bench with the pass chain as one captured graph (NDT_GRAPH=1, default) and as plain stream launches (0),
# then a kernel trace of each to see where the gaps between kernels sit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 1 0 1 0; do
  NDT_GRAPH=$g timeout -k 10 240 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/gab_$g.json 2> gpurun_out/gab_$g.err || { echo "bench $g failed"; tail -3 gpurun_out/gab_$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/gab_$g.json')); print('graph=$g', d['value'], d['ms_per_step'])"
done
for g in 1 0; do
  d=gpurun_out/gtr_$g; rm -rf $d
  NDT_GRAPH=$g timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $d.json 2> $d.err || { echo "trace $g failed"; exit 1; }
done
