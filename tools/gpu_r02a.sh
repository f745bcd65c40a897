#!/bin/bash
# Round-2 check: full-size parity tests, the C4 device-generated set (N=1 and through torchrun + RCCL at world 1), the
# default bench line with the BASELINE §3 CPU protocol.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1500 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 900 --timeout-method thread > $O/pytest_full.log 2>&1; rc=$?
echo "pytest full rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/pytest_full.log | head -20
[ $rc -ne 0 ] && { tail -40 $O/pytest_full.log; exit $rc; }
timeout -k 10 300 python bench.py --workload c4 --steps 64 --warmup 2 --no-cpu-baseline > $O/c4_64.json 2> $O/c4_64.err || { echo "c4 failed"; tail -20 $O/c4_64.err; exit 1; }
cat $O/c4_64.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --workload c4 --steps 32 --warmup 2 --no-cpu-baseline > $O/c4_trun.json 2> $O/c4_trun.err || { echo "c4 torchrun failed"; tail -20 $O/c4_trun.err; exit 1; }
cat $O/c4_trun.json
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
