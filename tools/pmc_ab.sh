#!/bin/bash
# PMC counter groups of one kernel for each library given (product libndt_hip.so or `make VARIANT=` builds):
# WL workload, KRE kernel regex.  One rocprofv3 run per counter group, never combined with tracing domains.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-c5}; STEPS=${STEPS:-3}; KRE=${KRE:-k_pass_(lead|direct)}
CGROUPS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_VMEM"
)
for lib in "$@"; do
  i=0
  for g in "${CGROUPS[@]}"; do
    i=$((i+1)); d=gpurun_out/pmcab/$WL/$lib/g$i; rm -rf $d; mkdir -p $d
    NDT_HIP_LIB=$lib timeout -k 10 -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "$KRE" -d $d -o run --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 1 --no-cpu-baseline > $d.out 2> $d.err || { echo "pmc $lib group $i failed"; tail -5 $d.err; exit 1; }
  done
  echo "== $lib"; python3 tools/pmc_summary.py gpurun_out/pmcab/$WL/$lib
done
