"""lorb_slam_amd -- MI355X-native LORB_SLAM matcher + local-BA hot path.

The product is liblorb.so (HIP/gfx950 kernels + C-ABI, include/lorb_c.h) and the C++ host
classes above it.  This package is thin Python plumbing over the C-ABI (ctypes), used by the
tests and bench.py.  See DESIGN.md.
"""
