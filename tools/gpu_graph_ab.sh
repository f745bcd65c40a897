set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for g in 1 0; do
  rm -rf gpurun_out/g$g
  NDT_GRAPH=$g timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/g$g -o run --output-format csv -- python3 bench.py --steps 12 --warmup 2 --no-cpu-baseline > gpurun_out/g$g.json 2> gpurun_out/g$g.err || exit 1
  echo "graph=$g"; python3 tools/trace_gaps.py gpurun_out/g$g/run_kernel_trace.csv
done
NOTEST=1 CFGS='c2;c2 NDT_GRAPH=0;c2;c2 NDT_GRAPH=0' bash tools/gpu_ab.sh
