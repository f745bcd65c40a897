set -o pipefail
TESTS='tests/test_gpu_parity.py tests/test_gpu_lead.py tests/test_gpu_fullsize.py::test_c5_full_size_res05 tests/test_gpu_fullsize.py::test_c2_full_size tests/test_gpu_fullsize.py::test_c4_batch_pairs_vs_oracle' bash tools/gpu_ab_micro.sh libndt_hip.so libndt_hip_notri.so libndt_hip_nopk.so || exit 1
for lib in libndt_hip.so libndt_hip_nolock.so libndt_hip_lockhi.so; do
  NDT_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload c4 --steps 512 --warmup 8 --no-cpu-baseline > gpurun_out/ab/c4_$lib.json 2> gpurun_out/ab/c4_$lib.err || { echo "c4 $lib failed"; tail -5 gpurun_out/ab/c4_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/c4_$lib.json')); r=d['roofline']; print('c4', '$lib', d['value'], r.get('ms_per_launch'), r.get('frac'), r.get('aggregate_frac'))"
done
WL=c5 LIB=libndt_hip_notri.so bash tools/gpu_pmc_micro.sh && WL=c5 bash tools/gpu_pmc_micro.sh
