#!/bin/bash
# Session A/B: GPU tests at the default build, pass-kernel micro A/B over variant libraries (tools/gpu_ab_micro.sh), then
# the C4 line with and without lockstep batching.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS="${TESTS:-tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_lead.py tests/test_gpu_fullsize.py tests/test_gpu_odom.py}" \
  bash tools/gpu_ab_micro.sh ${MICRO_LIBS:-libndt_hip.so} || exit 1
for lib in ${C4_LIBS:-libndt_hip.so libndt_hip_nolock.so}; do
  NDT_HIP_LIB=$lib timeout -k 10 400 python bench.py --workload c4 --steps ${C4_STEPS:-512} --warmup 8 --no-cpu-baseline > gpurun_out/ab/c4_$lib.json 2> gpurun_out/ab/c4_$lib.err || { echo "c4 $lib failed"; tail -5 gpurun_out/ab/c4_$lib.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/c4_$lib.json')); r=d['roofline']; print('c4', '$lib', d['value'], r.get('ms_per_launch'), r.get('frac'), r.get('aggregate_frac'))"
done
echo s1 done
