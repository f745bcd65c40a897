#!/bin/bash
# GPU tests (one process, stop at the first failure), then the rocprofv3 step timeline of the workloads in WLS
# (tools/gpu_trace_c2.sh) — the usual check after a change to the align / build path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_check.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_check.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/pytest_check.log | head -30; exit $rc; }
WLS=${WLS:-c2} bash tools/gpu_trace_c2.sh
