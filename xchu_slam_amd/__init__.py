"""xchu_slam_amd — MI355X-native NDT scan-matching path of lowmee/xchu_slam (odom_node's registration step).

Product = libndt_hip.so (HIP kernels for gfx950 behind the C-ABI in include/ndt_hip.h) + this thin
host mirror of the pclomp::NormalDistributionsTransform API.  See DESIGN.md.
"""
from .odom import LidarOdom  # noqa: F401
from .ndt import (DIRECT1, DIRECT7, DIRECT26, KDTREE, CpuNormalDistributionsTransform, NormalDistributionsTransform,  # noqa: F401
                  as_points, filter_scan, voxel_downsample)

__version__ = "0.1.0"
