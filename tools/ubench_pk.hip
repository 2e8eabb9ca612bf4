// Micro-benchmark: f32 multiply/add issue rate of plain VALU (v_mul_f32 /
// v_add_f32) against packed v_pk_mul_f32 / v_pk_add_f32 on gfx950, to decide
// whether the flat-list kernel (two triangles per lane per iteration as
// float2) can beat the unpacked issue ceiling.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/ubench_pk tools/ubench_pk.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int kChains>
__global__ void k_scalar(float* out, int iters, float a, float b) {
    float x[kChains];
    for (int c = 0; c < kChains; c++) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < kChains; c++) x[c] = x[c] * a + b;  // mul then add (contraction off)
    }
    float s = 0;
    for (int c = 0; c < kChains; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int kChains>
__global__ void k_packed(float* out, int iters, float a, float b) {
    f2 x[kChains];
    for (int c = 0; c < kChains; c++) x[c] = f2{threadIdx.x * 1e-3f + c, threadIdx.x * 2e-3f + c};
    const f2 av = f2{a, a}, bv = f2{b, b};
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < kChains; c++) x[c] = x[c] * av + bv;
    }
    float s = 0;
    for (int c = 0; c < kChains; c++) s += x[c].x + x[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 4096;
    float* out;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        float ms;
        hipEventRecord(e0);
        k_scalar<8><<<blocks, threads>>>(out, iters, 0.999f, 1e-4f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double ops = 2.0 * 8 * iters * (double)blocks * threads;
        printf("scalar: %.3f ms, %.1f T f32 ops/s\n", ms, ops / ms / 1e9);
        hipEventRecord(e0);
        k_packed<8><<<blocks, threads>>>(out, iters, 0.999f, 1e-4f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        ops = 2.0 * 2 * 8 * iters * (double)blocks * threads;
        printf("packed: %.3f ms, %.1f T f32 ops/s\n", ms, ops / ms / 1e9);
    }
    hipFree(out);
    return 0;
}
