#!/bin/bash
# Product GPU tests, then the split-accumulation library's parity tests and the single-pass A/B (c5, c2) against the product,
# then a C3 trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_prod.log 2>&1; rc=$?
echo "product pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_prod.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/pytest_prod.log | head -20; exit $rc; }
TESTS="tests/test_gpu_parity.py tests/test_gpu_lead.py tests/test_gpu_fullsize.py" TESTLIB=libndt_hip_split.so bash tools/gpu_ab_micro.sh libndt_hip.so libndt_hip_split.so || exit 1
bash tools/gpu_c3_trace.sh
