#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group; --pmc never combined with tracing domains).
# Usage: bash tools/pmc.sh <kernel-regex> [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
KRE=${1:-k_pass_(lead|direct)}
shift
ARGS=${@:---steps 10 --warmup 2 --no-cpu-baseline}
mkdir -p gpurun_out/pmc
CGROUPS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F64"
)
i=0
for g in "${CGROUPS[@]}"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc/g$i
  timeout -k 10 300 rocprofv3 --pmc $g --kernel-include-regex "$KRE" -d gpurun_out/pmc/g$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/g$i.out 2> gpurun_out/pmc/g$i.err || { echo "pmc group $i failed"; tail -5 gpurun_out/pmc/g$i.err; exit 1; }
done
echo "pmc done"
