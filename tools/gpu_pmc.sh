#!/bin/bash
# HBM traffic counters of the pass kernels at HEAD (FETCH_SIZE / WRITE_SIZE / L2 hit, one rocprofv3 pass per counter
# group, tools/pmc.sh) for C2 (k_pass_lead) and C5 (k_pass_direct), converted by tools/pmc_traffic.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc gpurun_out/pmc_c2 gpurun_out/pmc_c5
bash tools/pmc.sh 'k_pass_(lead|direct)' --steps 10 --warmup 2 --no-cpu-baseline || exit 1
mv gpurun_out/pmc gpurun_out/pmc_c2
bash tools/pmc.sh 'k_pass_(lead|direct)' --workload c5 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
mv gpurun_out/pmc gpurun_out/pmc_c5
python3 tools/pmc_traffic.py gpurun_out/pmc_c2 gpurun_out/pmc_traffic.json "tools/gpu_pmc.sh (tools/pmc.sh k_pass_(lead|direct), c2: k_pass_lead), ${PMC_LABEL:-round 6 HEAD}"
python3 tools/pmc_traffic.py gpurun_out/pmc_c5 gpurun_out/pmc_traffic_c5.json "tools/gpu_pmc.sh (tools/pmc.sh k_pass_(lead|direct) --workload c5: k_pass_direct), ${PMC_LABEL:-round 6 HEAD}"
echo pmc session done
