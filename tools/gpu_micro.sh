#!/bin/bash
# tools/pass_micro.py under rocprofv3 for each library given: single-pass kernel time (k_pass_direct) of WL.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${WL:-c5}; REPS=${REPS:-20}
for lib in "$@"; do
  d=gpurun_out/micro_${WL}_$lib; rm -rf $d
  NDT_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/pass_micro.py $WL $REPS > $d.out 2> $d.err || { echo "$lib failed"; tail -3 $d.err; exit 1; }
  echo "== $lib $(tail -1 $d.out)"
  python3 tools/kstats.py $d/run_kernel_stats.csv 1 | grep -E "k_pass"
done
