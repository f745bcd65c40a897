set -o pipefail
mkdir -p gpurun_out/dbg
NDT_HIP_LIB=libndt_hip_dbg.so timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dbg/c5.json 2> gpurun_out/dbg/c5.err || { tail -5 gpurun_out/dbg/c5.err; exit 1; }
NDT_HIP_LIB=libndt_hip_dbg.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/dbg/c2.json 2> gpurun_out/dbg/c2.err || { tail -5 gpurun_out/dbg/c2.err; exit 1; }
python3 -c "
import json
for w in ('c5','c2'):
    d=json.load(open('gpurun_out/dbg/%s.json'%w)); r=d['roofline']
    print(w, d['value'], r.get('ms_per_launch'), r.get('phases_ms'), r.get('workgroup_phases_ms'), r.get('tail_phases_ms'))
"
timeout -k 10 300 python -u -m pytest tests/test_gpu_odom.py -m gpu -q --timeout 200 --timeout-method thread -k "failure" 2>&1 | tail -3
