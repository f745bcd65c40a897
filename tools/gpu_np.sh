#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
NDT_HIP_LIB=libndt_hip_np.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q --timeout 300 --timeout-method thread > $O/pytest_np.log 2>&1; rc=$?
echo "pytest np rc=$rc"; tail -2 $O/pytest_np.log
[ $rc -ne 0 ] && { grep -E "FAIL|assert" $O/pytest_np.log | head; exit $rc; }
NOTEST=1 CFGS="c2;c2 NDT_HIP_LIB=libndt_hip_np.so;c2;c2 NDT_HIP_LIB=libndt_hip_np.so" bash tools/gpu_ab.sh
NDT_HIP_LIB=libndt_hip_dbgnp.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ph_c2.json 2> $O/ph_c2.err || exit 1
python -c "import json;d=json.load(open('$O/ph_c2.json'));r=d['roofline'];print('c2 np dbg',d['value'],r['ms_per_launch'],r['phases_ms'],r.get('tail_phases_ms'))"
