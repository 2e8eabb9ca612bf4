// rt_rcp.h -- the reciprocal the kFast walks take for 1 / r and 1 / f,
// shared by the kernels (rt_kernels_impl.h) and the exhaustive GPU check
// that licenses it (tools/check_rcp.hip, run by
// tests/test_gpu_parity.py::test_rcp_newton_exhaustive), so the check always
// tests the library's own code.
#pragma once
#include <hip/hip_runtime.h>

namespace rt {

// The correctly rounded 1.0f / x (the reference's 1 / r and (float)(1.0 /
// (double)f)) for |x| in [2^-126, 2^126): the hardware reciprocal and one
// Newton step with fused multiply-adds.  tools/check_rcp.hip compares it
// with the division bit for bit over every float of that range (both signs,
// 4.23e9 values, no difference on the MI355X: profiles/r05/check_rcp.json);
// callers take it only for waves whose operands all lie in the range.
__device__ __forceinline__ float rcp_nr(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, r, 1.0f);
    return fmaf(e, r, r);
}
__device__ __forceinline__ bool rcp_nr_ok(float x) { return fabsf(x) >= 0x1p-126f && fabsf(x) < 0x1p126f; }

}  // namespace rt
