// rt_internal.h -- shared between the host C++ (scene_host.cpp, rt_api.cpp)
// and the HIP kernels (rt_kernels.hip).  Device-side data layouts live here.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

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

// Per-pixel kernels: a block is a tile_w x 8 pixel tile made of 8x8-pixel
// wave64s (tile_w = 32 for the flat kernel, 16 for the KD kernel, whose LDS
// stack is three words per entry).
constexpr int kTileH = 8;
constexpr int kTileWFlat = 32;
constexpr int kTileWKd = 16;
constexpr int kBlockMax = 256;

// Interior record (64 B) of the KD layout: the two children's
// camera-relative boxes plus this node's split thresholds and child references.
//   r0 = (L.t0x, L.t1x, L.t0y, L.t1y)   r1 = (L.t0z, L.t1z, R.t0x, R.t1x)
//   r2 = (R.t0y, R.t1y, R.t0z, R.t1z)   r3 = (S_gt, S_lt, Lref | axis << 29, Rref | tiny_s1 << 29)
// (k_cam_nodes: S_gt / S_lt are the exact float forms of the reference's
// double tests against s2; s1 = L's high and s2 = R's low bound on the axis.)
constexpr uint32_t kRefMask = 0x1FFFFFFFu;
constexpr uint32_t kAxisShift = 29;
constexpr uint32_t kTinyS1Bit = 1u << 29;
// k_cam_nodes' flags of a camera's records
constexpr int32_t kCamTinyS1 = 1, kCamUnordered = 2;

// rt_camera_set_option keys.
enum Option : int32_t {
    kOptKernel = 1,     // KD kernel: 2 (per-lane DFS in the reference's order) or 3 (item pool, default)
    kOptTileOrder = 2,  // 0 XCD-contiguous, 1 natural, 2 centre-out, 3 by measured cost (kernel 3)
    kOptRays = 3,       // kernel 3 pixels per wave: 32, 16 or 8 (0 = auto)
    kOptItems = 4,      // kernel 3 items popped per lane per iteration: 1 or 2
    kOptCoarse = 5,     // kernel 3 coarse groups per wave outside the root box's rectangle (0 = off)
    kOptShadowOrder = 6,  // kernel 3 any-hit push order 0..3, -1 = timed choice (default)
    kOptFlat = 7,       // flat-list kernel: 9 one pass, 12 the list in 16 chunks (default)
    kOptRaysUsed = 8,   // get only: pixels per wave of the last kernel-3 render
    kOptSplitUsed = 9,  // get only: split tiles at the head of the current cost order (kernel 3)
    // 10, 11: retired (ABI 2; round 4's coop-used and frame-group keys)
    kOptFastUsed = 12,  // get only: which walks of the last kernel-3 render took the kFast forms (bit mask)
    kOptOrderRestores = 13,  // get only: kept cost orders restored (restore_order)
    kOptFineTiles = 14,  // get only: fine tiles (one kRays unit per wave) of the last kernel-3 render
    kOptDebug = 100,    // diagnostics: 1 = skip traversal, 2 = per-wave timestamps, 4 = every group
                        // coarse, 8 = coarse kernel on a side stream beside the fine one,
                        // 16 = counted shadow walks stop at occluders (the timed walk's work),
                        // 32 = counting renders stop after the root test, 64 = order / cost
                        // buffers sized for the current grid only, 256 = no held fine region,
                        // 512 = no split tiles, 1024 = no two-level iterations, 2048 = no kFast walks,
                        // 8192 = no clipped rectangle for a root box at the eye's depth,
                        // 16384 = record-load statistics (diagnostic builds, RT_VMEM_STATS)
    kOptPoolCap = 101,  // tests: shrink kernel 3's item pool (66..kPoolCap) to force its fallback
};
constexpr int kPoolCapMax = 640;

// Waves per block of the wave-cooperative kernel: a block is one fine tile,
// each wave one kRays-pixel unit of it.  16- and 8-ray units may run
// RT_KD3_WAVES per block (2 or 4; the tile's waves share the CU's L1), 32-
// and 64-ray units run 2.  The per-unit cost slots hold up to 4 waves.
#ifndef RT_KD3_WAVES
#define RT_KD3_WAVES 4
#endif
__host__ __device__ constexpr int kd3_waves(int rays) { return rays <= 16 ? RT_KD3_WAVES : 2; }
// Kernel 3's per-tile cost slots (pool iterations): slots 0-3 the waves of a
// tile, 4-7 the second half's waves of a split tile (zero otherwise), so a
// split tile's cost is the max over both halves, not whichever half wrote
// last (that race reordered the heavy tiles at random between samples).
constexpr int kCostSlots = 8;

// ---------------------------------------------------------------------------
// Device layouts (all 16-byte aligned, read with dwordx4 loads).
//
// Interior records: above (kRefMask, kAxisShift), camera-relative, one per
// interior node (init_cam_voxel_mem_cuda, TD/Camera.cu:137-162).
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
    const float4* tpair;           // flat variant 2: triangle pairs (k_pair_tri), or null
    const float4* shade;
    uint32_t* argb;
    int64_t* hit;
    // rt_render_display: the frame the reference's window shows
    // (TD/WinMain.cpp:212-237), or null: argb holds the previous frame's
    // clean buffer on entry; a hit pixel shows this frame's Phong, a miss
    // keeps the previous clean value (color_cam_cuda writes rmi >= 0 only)
    uint32_t* display;
    unsigned long long* counters;  // 5 x u64 or null
    int32_t* err;                  // device error word
    float n_mod[3], u_mod[3], v_mod[3];
    float xf[12];
    int32_t w, h;
    int32_t nranks, rank;
    int32_t frame_out;             // RT_FLAG_FRAME_OUT: tile pixels at their frame rows
    int32_t tiles_x, block_rows;   // fine grid = tiles_x * block_rows blocks
    // Fine region (kernel 3): the tiles covering the root box's screen
    // rectangle start at tile column fine_tx0 and band slot fine_s0; every
    // other 8x8 group of this rank's bands is a coarse group, handled
    // `coarse_per_wave` to a wave after the fine blocks (exact either way:
    // a coarse group runs the same root test and traces what passes).
    int32_t fine_tx0, fine_s0;
    int32_t groups_x, nslots;      // 8-px groups per row, band slots of this rank
    int32_t cg_x0, cg_x1;          // fine region in 8-px groups [x0, x1)
    int32_t cs0, cs1;              // fine region in slots [s0, s1)
    int32_t coarse_per_wave;       // coarse groups per wave
    int32_t any_order;             // push order of any-hit (shadow) walks 0..3, +4: counted walks stop at occluders
    int32_t coarse_blocks;         // blocks of k_coarse_kd3
    int32_t fill_blocks;           // blocks after the fine grid filling far groups (fused mode)
    int64_t coarse_groups;         // total coarse groups
    int32_t plain_xf;              // object transform is the identity (rotation 1, offset 0)
    // kernel 3's kFast walks apply (rt_api.cpp fast_proof): ordered boxes,
    // and every box's entry parameter >= 2^-20 for every ray of the frame
    // (any rotation; with an offset the translated walks take xfast_slot)
    int32_t fast;
    // shadow walks (round 6): the translated kFast slots apply to a shadow
    // ray that points to side sh_neg (1: negative) of axis sh_axis with
    // normal, nonzero components (rt_api.cpp fast_proof_shadow)
    int32_t fast_sh, sh_axis, sh_neg;
    uint32_t leaf_off;             // byte offset of trec from inode (one allocation; rt_api.cpp prepare_camera_object)
    uint32_t rec_bytes;            // bytes of that allocation's records (inode + trec; < 4 GiB when leaf_off is set)
    int32_t tiny_s1;               // some interior record of the camera has the tiny-s1 flag
    int32_t far_rect[4];           // root box's screen rectangle + 2 px (x0, x1, y0, y1; frame pixels)
    int32_t far_all;               // every group background: the box lies behind the eye (box_behind)
    int32_t tile_w, tile_h;        // pixels per block (tile_h divides the 8-row band)
    int32_t rays;                  // pixels (rays) per wave: 32, 16 or 8
    int32_t tile_order;            // Option kOptTileOrder
    const int32_t* order;          // tile permutation (tile_order 2: centre-out, 3: by cost)
    // kernel 3, tile order 3 (16- and 8-ray units): order[0..split) render as
    // two halves (2 blocks per tile)
    int32_t split;
    uint32_t* cost;                // tile_order 3: pool iterations per fine unit [tile][kCostSlots], or null
    float root_box[6];             // camera-relative root AABB (t0x,t1x,t0y,t1y,t0z,t1z)
    int32_t pool_cap;              // kernel 3 item-pool capacity in use (<= kPoolCap)
    int32_t items;                 // kernel 3 items per lane per iteration (1 or 2)
    int32_t debug;                 // diagnostic builds only: 1 = skip traversal
    unsigned long long* dbg;       // per-wave (t_start, t_end, visits) when non-null
    // diagnostic builds (-DRT_VMEM_STATS=1) with debug bit 16384: record-load
    // statistics per walk form (rt_kernels_impl.h vmem_stat), or null
    unsigned long long* vstat;
    // A multi-frame launch (kernel 3; pf_frames > 0): pf_frames frames of
    // pf_blocks blocks each in one grid, frame-major; frame f writes
    // pf_argb[(pf_seq0 + f) % pf_nbuf].
    int32_t pf_frames, pf_blocks, pf_seq0, pf_nbuf;
    uint32_t* pf_argb[RT_LOOP_MAX_BUF];
    uint32_t root_ref;
    uint32_t ntri;
    int32_t max_depth;
    int32_t tree_height;           // the scene tree's height (kernel 3's pool slack is height + 1)
    // kernel 3's two-level iterations: the deepest node depth whose children
    // are interior records at positions 2i + 1, 2i + 2 (-1: off)
    int32_t two_depth;
    int32_t flat_variant;          // Option kOptFlat: flat-list kernel form (9 or 12)
    // the chunked flat form (12, non-counting renders): per-pixel (w bits,
    // triangle) minima of the chunks, all ones between frames; and the chunk count
    unsigned long long* flat_key;
    int32_t flat_chunks;
};

// Blocks of k_trace_kd3's grid (fine tiles, split extras, far fill).
inline unsigned fine_grid_blocks(const TraceParams& p) {
    return (unsigned)(p.tiles_x * p.block_rows) + (unsigned)p.split + (unsigned)p.fill_blocks;
}

}  // namespace rt

// Kernel launchers (rt_kernels.hip), all stream-ordered.
namespace rt {
int launch_tri_world(const float* points9, const float* rad3, uint32_t ntri,
                     float4* tri_world, float4* shade, void* stream);
int launch_cam_tri(const float4* tri_world, uint32_t ntri, const float pos[3],
                   float4* trec, void* stream);
int launch_pair_tri(const float4* trec, uint32_t ntri, float4* tpair, void* stream);
int launch_cam_nodes(const rt_kd_node* nodes, const int32_t* interior_ids,
                     const uint32_t* node_ref, int64_t ninterior, const float pos[3],
                     float4* inode, int32_t* flags, void* stream);
// part: the coarse groups then the fine tiles (kPartAll), or one of them.
enum LaunchPart : int { kPartAll = 0, kPartFine = 1, kPartCoarse = 2 };
int launch_trace(const TraceParams& p, uint32_t mode, uint32_t flags, int kernel_version,
                 void* stream, int part);
// Camera-relative box of one world node, exactly as init_cam_voxel_mem_cuda.
void camera_relative_box(const rt_kd_node& nd, const float pos[3], float out[6]);
// KD build on the GPU (kd_build_gpu.hip).  The median tree's shape depends
// on the triangle count alone: per node its position range [l, r], median m,
// first child (-1 for a leaf) and parent; level k = nodes [level[k], level[k+1]).
struct KdShape {
    std::vector<int32_t> l, m, r, left, parent;
    std::vector<int64_t> level;
    int32_t height = 0;
};
void kd_shape(uint32_t n, KdShape& out);
// The node array of rt_kd_build, built on the current device into d_nodes
// (2n-1 entries); synchronises `stream`.
int kd_build_device(const rt_leaf_aabb* h_leafs, uint32_t n, const KdShape& shape, rt_kd_node* d_nodes, void* stream);
// Traversal refs: kLeafBit | tri for leaves, record position for interior ids.
int launch_node_ref(const rt_kd_node* d_nodes, int64_t nnode, const int32_t* d_ids, int64_t ninterior,
                    uint32_t* d_ref, void* stream);
// rt_kd_build's input checks: tri indices a permutation of [0, n), no NaN bound.
int validate_leafs(const rt_leaf_aabb* leafs, uint32_t n, const char* what);
int launch_unpack(int32_t w, int32_t h, int32_t nranks, const uint32_t* gathered,
                  uint32_t* frame, void* stream);
// Slots s of `rank` whose band rank + s*nranks lies in [b0, b1): [s0, s1).
__host__ __device__ inline void rect_slots(int32_t b0, int32_t b1, int32_t nranks, int32_t rank,
                                           int32_t& s0, int32_t& s1) {
    s0 = b0 <= rank ? 0 : (b0 - rank + nranks - 1) / nranks;
    s1 = b1 <= rank ? 0 : (b1 - 1 - rank) / nranks + 1;
    if (s1 < s0) s1 = s0;
}
// rect = (x0, x1, b0, b1): columns [x0, x1) of bands [b0, b1) (rt_frame_rect).
int launch_pack_rect(int32_t w, int32_t h, int32_t nranks, int32_t rank, const int32_t rect[4],
                     const uint32_t* local, uint32_t* out, void* stream);
int launch_unpack_rect(int32_t w, int32_t h, int32_t nranks, const int32_t rect[4], const uint32_t* local0,
                       const uint32_t* peers, uint32_t* frame, void* stream,
                       bool rect_only = false);
// rt_comm_gather_frame; rect_only: d_frame already holds this rectangle's
// background (an earlier gather of the same rectangle into it), so rank 0
// writes the rectangle alone.
int comm_gather_frame(rt_comm* c, rt_camera* cam, const float* xform, uint32_t mode, const uint32_t* d_local,
                      uint32_t* d_scratch, uint32_t* d_frame, void* stream, bool rect_only, int32_t rect_out[4]);
}  // namespace rt
