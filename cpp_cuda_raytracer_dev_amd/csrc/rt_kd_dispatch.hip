// rt_kd_dispatch.hip -- the KD kernels (k_trace_kd, k_trace_kd2,
// k_trace_kd3, k_coarse_kd3) of one (translated, write-hit, count)
// combination, selected by RT_KD_T / RT_KD_H / RT_KD_C (0 or 1); build.py
// compiles this file once per combination, in parallel.
// the header's other kernels (prep, flat, frame assembly) are launched from
// rt_kernels.hip; unused here
#pragma clang diagnostic ignored "-Wunused-function"
#include "rt_kernels_impl.h"

#if !defined(RT_KD_T) || !defined(RT_KD_H) || !defined(RT_KD_C)
#error "compile with -DRT_KD_T=0|1 -DRT_KD_H=0|1 -DRT_KD_C=0|1"
#endif

#define RT_CAT4(a, b, c, d) a##b##c##d
#define RT_NAME(t, h, c) RT_CAT4(kd_kernel_, t, h, c)

namespace rt {
TraceFn RT_NAME(RT_KD_T, RT_KD_H, RT_KD_C)(int version, int rays, int shadow, bool coarse) {
    return kd_kernel<RT_KD_T != 0, RT_KD_H != 0, RT_KD_C != 0>(version, rays, shadow, coarse);
}
}  // namespace rt
