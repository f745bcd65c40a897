#!/bin/bash
# PMC counter passes over tools/pass_micro.py (one derivative pass kernel, repeated): the load path (TA / TCP) and the
# SQ wave-state counters, one rocprofv3 --pmc pass per group.  Usage: WL=c5 LIB=libndt_hip.so bash tools/gpu_pmc_micro.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-c5}; LIB=${LIB:-libndt_hip.so}
O=gpurun_out/pmcm_${WL}_${LIB%.so}_${SET:-mem}; rm -rf $O; mkdir -p $O
if [ "${SET:-mem}" = lds ]; then
GROUPS_=(
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"
)
else
GROUPS_=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"
)
fi
i=0
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  NDT_HIP_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "k_pass" -d $O/g$i -o run --output-format csv -- python3 tools/pass_micro.py $WL 10 > $O/g$i.out 2> $O/g$i.err || { echo "pmc group $i failed"; tail -3 $O/g$i.err; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(O + "/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_pass" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print({k: round(tot[k] / n[k], 1) for k in sorted(tot)})
PY
