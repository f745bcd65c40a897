#!/bin/bash
# Per-phase timing of the derivative pass (profiling build with per-workgroup stamps) on C2 and C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
NDT_HIP_LIB=libndt_hip_dbg.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ph_c2.json 2> $O/ph_c2.err || { tail -20 $O/ph_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/ph_c2.json'));r=d['roofline'];print('c2',d['value'],r['ms_per_launch'],r.get('phases_ms'),r.get('workgroup_phases_ms'),r.get('tail_phases_ms'))"
NDT_HIP_LIB=libndt_hip_dbg.so timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/ph_c5.json 2> $O/ph_c5.err || { tail -20 $O/ph_c5.err; exit 1; }
python -c "import json;d=json.load(open('$O/ph_c5.json'));r=d['roofline'];print('c5',d['value'],r['ms_per_launch'],r.get('phases_ms'),r.get('workgroup_phases_ms'),r.get('tail_phases_ms'))"
