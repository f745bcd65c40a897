set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
NDT_HIP_LIB=libndt_hip_dbg.so timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/dbg.json 2> gpurun_out/dbg.err && echo dbg ok &&
timeout -k 10 400 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err && echo c5 ok &&
timeout -k 10 500 python bench.py --workload c3 --steps 1000 --warmup 5 --no-cpu-baseline > gpurun_out/c3.json 2> gpurun_out/c3.err && echo c3 ok
