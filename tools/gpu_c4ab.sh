#!/bin/bash
# C4 batched replay A/B over stream counts, the per-stream CU share and the HIP hardware-queue count (256 pairs each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-"NDT_BATCH_STREAMS=3 NDT_BATCH_SHARE=1"}
IFS=';' read -ra CL <<< "$CFGS"
for cfg in "${CL[@]}"; do
  env $cfg timeout -k 10 300 python bench.py --workload c4 --steps 256 --warmup 4 --no-cpu-baseline > gpurun_out/c4ab.json 2> gpurun_out/c4ab.err || { echo "$cfg failed"; tail -5 gpurun_out/c4ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c4ab.json'));print('$cfg', d['value'], d['ms_per_step'], d['mean_translation_error_m'])"
done
