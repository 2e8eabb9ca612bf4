"""MI355X-native per-pixel ray caster: a drop-in for the hot path of
ams3878/cpp_cuda_raytracer_dev (primary rays -> KD traversal ->
Moller-Trumbore -> Phong -> u32 frame), as hand-written gfx950 HIP kernels
behind a C ABI (include/rt_mi355x.h).

The HIP library is loaded lazily by the submodules that need it; there is no
CPU fallback in this package.
"""
__version__ = "0.1.0"
