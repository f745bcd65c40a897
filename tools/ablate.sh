#!/bin/bash
# Build pass-kernel ablation variants (experiment only) into build/ablate/<v>/libndt_hip.so
set -e
cd "$(dirname "$0")/.."
# VARIANTS="name:-DFLAG ..." overrides the default ablation set (0..3)
VARIANTS=${VARIANTS:-"0:-DNDT_ABLATE=0 1:-DNDT_ABLATE=1 2:-DNDT_ABLATE=2 3:-DNDT_ABLATE=3"}
for vv in $VARIANTS; do
  v=${vv%%:*}; flags=${vv#*:}; flags=${flags//,/ }
  d=build/ablate/$v; mkdir -p $d/obj
  for f in voxel_build derivatives solver front_end ndt_api; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags -c xchu_slam_amd/csrc/$f.hip -o $d/obj/$f.o &
  done
  g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c xchu_slam_amd/csrc/odom_estimate.cpp -o $d/obj/odom_estimate.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libndt_hip.so $d/obj/*.o
done
