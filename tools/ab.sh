#!/bin/bash
# The A/B driver: rocprofv3 kernel statistics + bench value of one workload (WL, STEPS) for each library given as an
# argument (libndt_hip.so = product, libndt_hip_<name>.so = `make -C xchu_slam_amd/csrc VARIANT=<name> VFLAGS=-D...`
# builds of a candidate change); KERN filters the kernel lines.  Single-pass kernel A/B: tools/gpu_micro.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${WL:-c5}; STEPS=${STEPS:-5}; KERN=${KERN:-.}
for lib in "$@"; do
  d=gpurun_out/lab_${WL}_$lib; rm -rf $d
  NDT_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --workload $WL --steps $STEPS --warmup 2 --no-cpu-baseline > $d.json 2> $d.err || { echo "$lib failed"; tail -3 $d.err; exit 1; }
  echo "== $WL $lib $(python3 -c "import json; d=json.loads(open('$d.json').read().strip().splitlines()[-1]); print(d['value'], d.get('breakdown_ms_per_step'))")"
  python3 tools/kstats.py $d/run_kernel_stats.csv $((STEPS+2)) > $d.txt; grep -E "$KERN" $d.txt
done
