// Exhaustive check (GPU) that the reciprocal kFast walks may use,
//   r = v_rcp_f32(x); e = fma(-x, r, 1); y = fma(e, r, r)
// equals the correctly rounded 1.0f / x (the library's division: hipcc
// -fhip-fp32-correctly-rounded-divide-sqrt) bit for bit, for every float x
// with a normal magnitude in [2^-126, 2^126) of either sign.  Prints one JSON
// line: mismatches per binade and in total; exit 0 when there are none.
// Built in-tree by cpp_cuda_raytracer_dev_amd/build.py (tools/check_rcp),
// run by tests/test_gpu_parity.py::test_rcp_newton_exhaustive.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "rt_rcp.h"  // the library's rcp_nr itself

using rt::rcp_nr;

__global__ void k_check(uint32_t lo_exp, unsigned long long* bad_per_exp, uint32_t* first_bad) {
    // one thread per (sign, exponent, mantissa): grid-stride over 2 * n_exp * 2^23
    const uint64_t n_exp = 252;  // biased exponents 1 .. 252 (2^-126 .. 2^126)
    const uint64_t total = 2ull * n_exp << 23;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t m = (uint32_t)(i & ((1u << 23) - 1));
        const uint32_t e = lo_exp + (uint32_t)((i >> 23) % n_exp);
        const uint32_t sgn = (uint32_t)((i >> 23) / n_exp) << 31;
        const float x = __uint_as_float(sgn | (e << 23) | m);
        const float a = 1.0f / x;
        const float b = rcp_nr(x);
        if (__float_as_uint(a) != __float_as_uint(b)) {
            atomicAdd(&bad_per_exp[e], 1ull);
            atomicCAS(first_bad, 0u, __float_as_uint(x));
        }
    }
}

int main() {
    unsigned long long* d_bad;
    uint32_t* d_first;
    if (hipMalloc(&d_bad, 256 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&d_first, sizeof(uint32_t)) != hipSuccess)
        return 2;
    (void)hipMemset(d_bad, 0, 256 * sizeof(unsigned long long));
    (void)hipMemset(d_first, 0, sizeof(uint32_t));
    k_check<<<8192, 256>>>(1, d_bad, d_first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long bad[256];
    uint32_t first = 0;
    (void)hipMemcpy(bad, d_bad, sizeof bad, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&first, d_first, sizeof first, hipMemcpyDeviceToHost);
    unsigned long long total = 0;
    printf("{\"checked\": %llu, \"bad_by_biased_exponent\": {", 2ull * 252ull << 23);
    bool sep = false;
    for (int e = 0; e < 256; e++)
        if (bad[e]) {
            printf("%s\"%d\": %llu", sep ? ", " : "", e, bad[e]);
            sep = true;
            total += bad[e];
        }
    printf("}, \"bad\": %llu, \"first_bad_bits\": \"0x%08x\"}\n", total, first);
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    return total ? 1 : 0;
}
