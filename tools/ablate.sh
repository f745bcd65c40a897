#!/bin/bash
# Build pass-kernel ablation variants (experiment only) into build/ablate/<v>/libndt_hip.so
set -e
cd "$(dirname "$0")/.."
for v in 0 1 2 3; do
  d=build/ablate/$v; mkdir -p $d/obj
  for f in voxel_build derivatives solver ndt_api; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DNDT_ABLATE=$v -c xchu_slam_amd/csrc/$f.hip -o $d/obj/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libndt_hip.so $d/obj/*.o
done
