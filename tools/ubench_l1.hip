// tools/ubench_l1.hip -- design tool (not product, not a test): what one
// wave-wide 16-byte-per-lane load costs the CU's vector memory path on the
// MI355X as a function of how its 64 lanes' addresses share 128-byte lines
// (verdict r05 item 1: k_trace_kd3's texture data unit is busy on 0.96 of CU
// cycles, and TCP_TOTAL_CACHE_ACCESSES runs at ~0.94 per CU cycle).
//
// Every wave loops over an L1-resident 16 KiB table (128 lines of 128 B) and
// issues kLoads independent global_load_dwordx4 per iteration before it
// consumes them, as the walk does with a record.  The pattern fixes, per
// instruction, which line and which 16-byte quarter each lane reads:
//   0  64 lines, one 16-B piece each (lane-per-record, records in distinct lines)
//   1  16 lines, 4 consecutive lanes read the 4 quarters of one 64-B half
//   2  16 lines, lanes l, l+16, l+32, l+48 share a line (non-adjacent sharers)
//   3   8 lines, 8 consecutive lanes read one whole 128-B line
//   4   1 line, every lane the same 16 B
//   5  16 lines, 4 consecutive lanes read the SAME 16 B (four rays at one node)
//   6  32 lines, lanes 2k, 2k+1 read the two 64-B halves' first quarters
//      (sibling records sharing a line)
//   7  64 lines, as 0, but only lanes < 16 active (exec-masked loads)
//   8  16 lines as 5 but the sharers spread (lane l reads line l % 16)
//   9  buffer loads: lane 4k reads its own line, lanes 4k+1..4k+3 an offset
//      beyond the buffer's range (the range check drops them)
//  10  buffer loads, every lane its own line (pattern 0 through a buffer)
//  11  global loads exec-masked to lane 4k (one lane per quad, own lines)
//  12  16 lines, lane 4k's line shared by its quad but lanes 4k+1..4k+3 are
//      exec-masked (the leader-only form of pattern 5)
// Prints one JSON line per pattern: ns per wave-instruction per CU, and
// cycles at the measured shader clock (s_memtime against s_memrealtime).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_l1 tools/ubench_l1.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kLines = 128;      // 16 KiB table
constexpr int kLoads = 4;        // independent loads in flight per iteration
constexpr int kIters = 2048;

template <int kPat>
__device__ __forceinline__ uint32_t offset_of(int lane, int it, int k, int wave) {
    const int rot = (it * kLoads + k + wave * 5) & (kLines - 1);  // a different set of lines each instruction
    int line = 0, byte = 0;
    switch (kPat) {
    case 0: line = lane; byte = 0; break;
    case 1: line = lane >> 2; byte = (lane & 3) * 16; break;
    case 2: line = lane & 15; byte = (lane >> 4) * 16; break;
    case 3: line = lane >> 3; byte = (lane & 7) * 16; break;
    case 4: line = 0; byte = 0; break;
    case 5: line = lane >> 2; byte = 0; break;
    case 6: line = lane >> 1; byte = (lane & 1) * 64; break;
    case 7: line = lane; byte = 0; break;
    case 8: line = lane & 15; byte = 0; break;
    }
    return (uint32_t)(((line + rot) & (kLines - 1)) * 128 + byte);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int kPat>
__global__ __launch_bounds__(256) void k_l1(const uint4* __restrict__ table, uint32_t* out, unsigned long long* clk) {
    const int lane = threadIdx.x & 63, wave = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    const char* base = (const char*)table;
    uint32_t acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)table, (short)0, kLines * 128, 0x00020000);
    for (int it = 0; it < kIters; it++) {
        uint4 v[kLoads];
        if ((kPat == 7 && lane >= 16) || ((kPat == 11 || kPat == 12) && (lane & 3) != 0)) {
            for (int k = 0; k < kLoads; k++) v[k] = make_uint4(0, 0, 0, 0);
        } else if (kPat == 9 || kPat == 10) {
#pragma unroll
            for (int k = 0; k < kLoads; k++) {
                const int off = (kPat == 9 && (lane & 3) != 0) ? 0x40000000 : (int)offset_of<0>(lane, it, k, wave);
                const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
                v[k] = make_uint4(r.x, r.y, r.z, r.w);
            }
        } else {
#pragma unroll
            for (int k = 0; k < kLoads; k++)
                v[k] = *(const uint4*)(base + offset_of<kPat == 11 ? 0 : kPat == 12 ? 5 : kPat>(lane, it, k, wave));
        }
#pragma unroll
        for (int k = 0; k < kLoads; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        acc = (acc << 1) | (acc >> 31);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (acc == 0x9e3779b9u) out[0] = acc;  // (never: keeps the loads)
    if (wave == 0 && lane == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int kPat>
void run(const uint4* table, uint32_t* out, unsigned long long* clk, int blocks, hipEvent_t e0, hipEvent_t e1) {
    for (int rep = 0; rep < 2; rep++) {  // the first launch warms the L1s
        hipEventRecord(e0);
        k_l1<kPat><<<blocks, 256>>>(table, out, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    const double ghz = h[1] ? (double)h[0] / ((double)h[1] * 10.0) : 0.0;  // s_memrealtime runs at 100 MHz
    const double instr_per_cu = (double)blocks * 4 * kIters * kLoads / 256.0;
    const double ns = ms * 1e6 / instr_per_cu;
    printf("{\"pattern\": %d, \"blocks\": %d, \"ms\": %.4f, \"ns_per_wave_load_per_cu\": %.3f, \"shader_ghz\": %.3f, "
           "\"cycles_per_wave_load_per_cu\": %.2f}\n",
           kPat, blocks, ms, ns, ghz, ns * ghz);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 256 * 6;  // 6 blocks of 4 waves per CU
    uint4* table;
    uint32_t* out;
    unsigned long long* clk;
    hipMalloc(&table, kLines * 128);
    hipMemset(table, 0x5a, kLines * 128);
    hipMalloc(&out, 4);
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    run<0>(table, out, clk, blocks, e0, e1);
    run<1>(table, out, clk, blocks, e0, e1);
    run<2>(table, out, clk, blocks, e0, e1);
    run<3>(table, out, clk, blocks, e0, e1);
    run<4>(table, out, clk, blocks, e0, e1);
    run<5>(table, out, clk, blocks, e0, e1);
    run<6>(table, out, clk, blocks, e0, e1);
    run<7>(table, out, clk, blocks, e0, e1);
    run<8>(table, out, clk, blocks, e0, e1);
    run<9>(table, out, clk, blocks, e0, e1);
    run<10>(table, out, clk, blocks, e0, e1);
    run<11>(table, out, clk, blocks, e0, e1);
    run<12>(table, out, clk, blocks, e0, e1);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        printf("error %s\n", hipGetErrorString(e));
        return 1;
    }
    return 0;
}
