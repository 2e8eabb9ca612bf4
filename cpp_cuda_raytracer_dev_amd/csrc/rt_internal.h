// rt_internal.h -- shared between the host C++ (scene_host.cpp, rt_api.cpp)
// and the HIP kernels (rt_kernels.hip).  Device-side data layouts live here.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_mi355x.h"

namespace rt {

// Error plumbing for rt_last_error_string (thread-local message).
int fail(int code, const char* fmt, ...);

// Leaf references in the traversal: a set top bit means "leaf; the low bits
// are a triangle index", otherwise the low bits index the dense interior-node
// array.  Trees are limited to < 2^31 triangles.
constexpr uint32_t kLeafBit = 0x80000000u;

// Traversal stack entries per lane kept in LDS.  The reference sizes the
// per-pixel stack ceil(log2(nvox)) (TD/Camera.cpp:202-203), which is exactly
// the maximum DFS occupancy of its balanced median tree; 24 covers 2^23 tris.
constexpr int kMaxDepth = 24;

// Threads per block for the per-pixel kernels: a 32x8 pixel tile, four
// wave64s of 8x8 pixels each.
constexpr int kTileW = 32;
constexpr int kTileH = 8;
constexpr int kBlock = kTileW * kTileH;

// ---------------------------------------------------------------------------
// Device layouts (all 16-byte aligned, read with dwordx4 loads).
//
// InteriorNode (48 B), camera-relative, one per interior node of the tree in
// BFS order (init_cam_voxel_mem_cuda, TD/Camera.cu:137-162):
//   a = (t0x, t1x, t0y, t1y)   d_Bo = h_bound - camera position
//   b = (t0z, t1z, s1, s2)     split planes minus camera[axis]
//   c = (left_ref, right_ref, axis, s1_eps_bits)
//        s1_eps = (float)((double)s1 + 1e-16), used when the object
//        translation is zero (TD/Trixel.cu:150 with ds == 0).
//
// TriRecord (64 B), camera-relative, one per triangle, indexed by
// tri_list_index (init_tri_mem_cuda + init_cam_tri_mem_cuda,
// TD/Trixel.cu:11-36):
//   (e1x, e1y, e1z, e2x) (e2y, e2z, dtx, dty) (dtz, dqx, dqy, dqz) (dw, 0, 0, 0)
//
// Shade (32 B), one per triangle: (nx, ny, nz, 0) (r, g, b, 0)
// ---------------------------------------------------------------------------

struct TraceParams {
    const float4* inode;
    const float4* trec;
    const float4* shade;
    uint32_t* argb;
    int64_t* hit;
    unsigned long long* counters;  // 5 x u64 or null
    int32_t* err;                  // device error word
    float n_mod[3], u_mod[3], v_mod[3];
    float xf[12];
    int32_t w, h;
    int32_t nranks, rank;
    int32_t tiles_x, slots;        // grid = tiles_x * slots blocks
    uint32_t root_ref;
    uint32_t ntri;
    int32_t max_depth;
};

}  // namespace rt

// Kernel launchers (rt_kernels.hip), all stream-ordered.
namespace rt {
int launch_tri_world(const float* points9, const float* rad3, uint32_t ntri,
                     float4* tri_world, float4* shade, void* stream);
int launch_cam_tri(const float4* tri_world, uint32_t ntri, const float pos[3],
                   float4* trec, void* stream);
int launch_cam_nodes(const rt_kd_node* nodes, const int32_t* interior_ids,
                     const uint32_t* node_ref, int64_t ninterior, const float pos[3],
                     float4* inode, void* stream);
int launch_trace(const TraceParams& p, uint32_t mode, uint32_t flags, void* stream);
int launch_unpack(int32_t w, int32_t h, int32_t nranks, const uint32_t* gathered,
                  uint32_t* frame, void* stream);
}  // namespace rt
