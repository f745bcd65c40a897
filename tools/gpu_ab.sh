#!/bin/bash
# GPU session: gpu tests (NOTEST=1 skips them), then short bench lines of the workloads in CFGS (';'-separated
# "workload [ENV=VAL ...]" entries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
fi
# CFGS: ';'-separated "workload [ENV=VAL ...]" entries
CFGS=${CFGS:-"c2;c2 NDT_SOURCE_ORDER=0;c5;c5 NDT_SOURCE_ORDER=0"}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for cfg in "${CFG_LIST[@]}"; do
  set -- $cfg; wl=$1; shift
  name=$(echo "$cfg" | tr ' =/.' '____')
  steps=30; [ "$wl" = "c5" ] && steps=5
  env "$@" timeout -k 10 300 python bench.py --workload $wl --steps $steps --warmup 2 --no-cpu-baseline > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "bench $cfg failed"; tail -5 gpurun_out/ab_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], d.get('breakdown_ms_per_step'), r['ms_per_launch'], r['frac'])"
done
