// rt_kernels_impl.h -- gfx950 kernels of the per-pixel ray-cast hot path
// (included by rt_kernels.hip and, once per (translated, write-hit, count)
// combination, by rt_kd_dispatch.hip, so the KD kernels' many template
// instances compile in parallel translation units).
//
// One fused kernel per frame: primary ray -> object transform -> KD-tree
// traversal (or the flat triangle list) -> Moller-Trumbore -> Phong -> u32
// 0x00RRGGBB.  The KD path's kernel is k_trace_kd3: a wave pools the (ray,
// node) items of its 8/16/32 rays in an LDS stack and every lane visits any
// ray's item, with ballot / mbcnt compaction of the pushed children and a
// 64-bit LDS minimum of (w, DFS path code) for the reference's tie rule.
// k_trace_kd2 is the per-lane DFS in the reference's visiting order (its
// counters are the reference's, bench.py's counting frame).  Blocks take
// screen tiles in a cost-ordered permutation the host keeps.
//
// Arithmetic follows the reference expression by expression (SURVEY.md §5
// H1-H16): single precision with contraction off (-ffp-contract=off), the
// reference's double-promoted epsilons evaluated in double, correctly
// rounded float division (equal to the reference's (float)(1.0/f)), the
// 21-step fast inverse square root, and the deterministic pow5 shared with the
// oracle.  Every kernel cites the reference code it replaces.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "rt_internal.h"
#include "rt_predicates.h"
#include "rt_rcp.h"

namespace rt {
namespace {

constexpr double kEps = 1e-16;                  // TD/vector.cuh:10-11 (double literals)
// Smallest float >= 1e-16: for a float x, (double)x < 1e-16 <=> x < kEpsF and
// (double)x > -1e-16 <=> x > -kEpsF (1e-16 is not a float).  Checked in tests.
constexpr float kEpsF = __builtin_bit_cast(float, 0x24e69595u);
constexpr float kDrawDistance = 400.0f;         // TD/Trixel.cu:47
constexpr uint32_t kBackground = 0x00F08200u;   // VEC4<T_uint>(240,130,0,0), TD/Camera.cpp:72
constexpr uint32_t kMiss = 0xFFFFFFFFu;

// The wave's index in its block, as a scalar (the compiler cannot see that
// threadIdx.x >> 6 is wave-uniform and would keep it, and everything derived
// from it, in vector registers).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); }

// device_inverse_sqrt, TD/vector.cuh:79-95 (seed from bits(s/2), 21 steps).
__device__ __forceinline__ float rsqrt21(float x, float y, float z) {
    float s = (x * x) + (y * y) + (z * z);
    const float half = 0.5f * s;
    uint32_t i = 0x5f375a86u - (__float_as_uint(half) >> 1);
    float r = __uint_as_float(i);
#pragma unroll
    for (int k = 0; k < 21; k++) r = r * (1.5f - half * r * r);
    return r;
}

// rcp_nr / rcp_nr_ok: rt_rcp.h (shared with tools/check_rcp.hip)

// device_cross / device_dot, TD/vector.cuh:72-77,121-124
__device__ __forceinline__ void cross3(float& cx, float& cy, float& cz, float ax, float ay,
                                       float az, float bx, float by, float bz) {
    cx = ay * bz - az * by;
    cy = az * bx - ax * bz;
    cz = ax * by - ay * bx;
}
__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return (ax * bx) + (ay * by) + (az * bz);
}

// powf(|x|, 5) of TD/Camera.cu:45 as one deterministic rounding (H5).
__device__ __forceinline__ float pow5(float x) {
    double d = (double)x;
    double d2 = d * d;
    double d4 = d2 * d2;
    return (float)(d4 * d);
}

// (u8)(float) with NaN -> 0 (H14).
__device__ __forceinline__ uint32_t to_u8(float t) {
    if (!(t >= 0.0f)) return 0u;
    if (t >= 256.0f) return 255u;
    return (uint32_t)(int)t;
}

// color_cam_cuda, TD/Camera.cu:27-60 (norm.x used twice in the dot, H1).
__device__ __forceinline__ uint32_t phong(const float pnt[3], const float nrm[3], const float rmd[3],
                          const float rad[3]) {
    float sdx = 2 - pnt[0], sdy = 2 - pnt[1], sdz = 2 - pnt[2];
    const float r = rsqrt21(sdx, sdy, sdz);
    sdx *= r; sdy *= r; sdz *= r;
    const float dot_r_n = dot3(sdx, sdy, sdz, nrm[0], nrm[0], nrm[2]);
    const float rx = (sdx - (2 * dot_r_n * nrm[0])) * rmd[0];
    const float ry = (sdy - (2 * dot_r_n * nrm[1])) * rmd[1];
    const float rz = (sdz - (2 * dot_r_n * nrm[2])) * rmd[2];
    const float diff = (float)(.6 * (double)fabsf(dot_r_n));
    const float spec = (float)((double)pow5(fabsf((rx + ry + rz))) * .3);
    float pr = 0.0f, pg = 0.0f, pb = 0.0f;
    pr += (rad[0] * diff) + (1 * spec);
    pg += (rad[1] * diff) + (1 * spec);
    pb += (rad[2] * diff) + (1 * spec);
    const float mx = fmaxf(fmaxf(pr, pg), pb);
    return (to_u8((pr / mx) * 255) << 16) | (to_u8((pg / mx) * 255) << 8) | to_u8((pb / mx) * 255);
}

// A pixel's frame write.  With P.display (rt_render_display) it also writes
// the reference's displayed frame: the clean buffer argb still holds the
// previous frame, which a miss keeps on screen (ghosting under motion: the
// window's buffer is overwritten by color_cam_cuda only where rmi >= 0,
// TD/Camera.cu:27-61, and reset to background + Phong by the SET pass after
// the blit, TD/WinMain.cpp:212-237, TD/Camera.cu:77-84).
// A multi-frame launch's output buffer of the frame a block renders
// (k_trace_kd3; stored by each wave's lane 0 at the block's start).
__shared__ uint32_t* s_pf_argb;

__device__ __forceinline__ void put_pixel(const TraceParams& P, int64_t out, uint32_t argb, bool hit) {
    if (P.display) P.display[out] = hit ? argb : P.argb[out];
    uint32_t* base = P.pf_frames > 0 ? s_pf_argb : P.argb;
    base[out] = argb;
}

// Block -> tile.  Order 0: blocks b and b+8 share an XCD, so give each XCD a
// contiguous run of tiles (bijective for any grid size); order 1: natural
// (neighbouring tiles on different XCDs); order 2: the host's centre-out
// permutation, so the heavy centre tiles are dispatched first; order 3: the
// host's permutation by the tiles' measured cost in an earlier frame,
// heaviest first (centre-out until costs arrive); order 4: the same per XCD
// over 8 screen regions of equal cost; order 5: per XCD over 8 row bands of
// equal tile count (rt_api.cpp cost_order).
__device__ __forceinline__ int32_t tile_index(const TraceParams& P, int32_t b) {
    const int32_t nblocks = P.tiles_x * P.block_rows;
    if (P.tile_order == 0) {
        const int32_t q = nblocks >> 3, rem = nblocks & 7;
        const int32_t xcd = b & 7, k = b >> 3;
        return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + k;
    }
    if (P.tile_order >= 2 && P.order) return P.order[b];  // orders 2-4: host permutation
    return b;
}

__device__ __forceinline__ void tile_of(const TraceParams& P, int32_t b, int32_t& tx, int32_t& slot) {
    const int32_t t = tile_index(P, b);
    slot = t / P.tiles_x;
    tx = t - slot * P.tiles_x;
    tx += P.fine_tx0;
    slot += P.fine_s0 * (kTileH / P.tile_h);
}

struct Pixel {
    int32_t x, y;      // frame coordinates (row 0 = bottom, TD/WinMain.cpp:32)
    int64_t out;       // index into the (packed) output buffer
};

// Tile b covers tile_w x tile_h pixels of one 8-row band; wave `wave` of it
// owns an 8 x (rays/8) sub-tile (side by side when tile_w > 8, stacked
// otherwise).  Lanes >= rays own no pixel (the wave-cooperative kernel's
// helper lanes).
// A wave's unit of pixels: 8 columns from x0, rows yin.. of band slot `slot`.
struct Unit {
    int32_t x0, slot, yin;
};

// Lane `lane`'s pixel of a unit (8 pixels per row, row-major); lanes >= rows*8
// own no pixel, nor do lanes whose column is >= cols (a split 8-ray unit's
// 4-pixel half).
__device__ __forceinline__ bool unit_pixel(const TraceParams& P, const Unit& u, int32_t rows, int32_t lane,
                                           Pixel& px, int32_t cols = 8) {
    const int32_t band = P.rank + u.slot * P.nranks;
    const int32_t ly = u.yin + (lane >> 3);
    px.x = u.x0 + (lane & 7);
    px.y = band * kTileH + ly;
    px.out = (int64_t)((P.frame_out ? band : u.slot) * kTileH + ly) * P.w + px.x;
    return lane < rows * 8 && (lane & 7) < cols && px.x < P.w && px.y < P.h;
}

// Sub-tile `wave` of the fine tile with index t (in the fine grid).
__device__ __forceinline__ Unit unit_of_tile(const TraceParams& P, int32_t t, int32_t wave) {
    int32_t row = t / P.tiles_x;
    const int32_t tx = t - row * P.tiles_x + P.fine_tx0;
    row += P.fine_s0 * (kTileH / P.tile_h);
    const int32_t per_band = kTileH / P.tile_h;
    const int32_t slot = row / per_band, yin = (row - slot * per_band) * P.tile_h;
    const int32_t wrows = P.rays >> 3;
    const int32_t wx = P.tile_w > 8 ? wave * 8 : 0, wy = P.tile_w > 8 ? 0 : wave * wrows;
    return Unit{tx * P.tile_w + wx, slot, yin + wy};
}

// Sub-tile `wave` of fine tile b.
__device__ __forceinline__ Unit unit_of(const TraceParams& P, int32_t b, int32_t wave) {
    int32_t tx, row;
    tile_of(P, b, tx, row);
    const int32_t per_band = kTileH / P.tile_h;
    const int32_t slot = row / per_band, yin = (row - slot * per_band) * P.tile_h;
    const int32_t wrows = P.rays >> 3;
    const int32_t wx = P.tile_w > 8 ? wave * 8 : 0, wy = P.tile_w > 8 ? 0 : wave * wrows;
    return Unit{tx * P.tile_w + wx, slot, yin + wy};
}

__device__ __forceinline__ bool pixel_of(const TraceParams& P, int32_t b, int32_t wave, Pixel& px) {
    return unit_pixel(P, unit_of(P, b, wave), P.rays >> 3, (int32_t)threadIdx.x & 63, px);
}

// Coarse group j (row-major over this rank's slots and 8-px columns, skipping
// the fine region) -> its 8x8 unit.  32-bit arithmetic: the host keeps
// coarse_groups below 2^31 (64-bit division is a long software sequence).
__device__ __forceinline__ Unit coarse_unit(const TraceParams& P, int32_t j) {
    const int32_t gx = P.groups_x;
    const int32_t before = P.cs0 * gx;
    int32_t slot, col;
    if (j < before) {
        slot = j / gx;
        col = j - slot * gx;
    } else {
        j -= before;
        const int32_t m = gx - (P.cg_x1 - P.cg_x0);
        const int32_t mid = (P.cs1 - P.cs0) * m;
        if (j < mid) {
            const int32_t r = j / m;
            slot = P.cs0 + r;
            col = j - r * m;
            if (col >= P.cg_x0) col += P.cg_x1 - P.cg_x0;
        } else {
            j -= mid;
            const int32_t r = j / gx;
            slot = P.cs1 + r;
            col = j - r * gx;
        }
    }
    return Unit{col * 8, slot, 0};
}

// One tile per block (blockIdx), one sub-tile per wave.
__device__ __forceinline__ bool pixel_of_thread(const TraceParams& P, Pixel& px) {
    return pixel_of(P, (int32_t)blockIdx.x, wave_id(), px);
}

// init_cam_mem_cuda, TD/Camera.cu:103-104: rmd = n + u*ix + v*iy, normalised.
// kR: the normalisation factor is given (rn, computed by an earlier call for
// the same pixel) instead of computed; else it is returned in rn.
template <bool kR = false>
__device__ __forceinline__ void primary_ray(const TraceParams& P, int32_t ix, int32_t iy,
                                            float rmd[3], float& rn) {
    // (float)ix of the reference's unsigned pixel index: exact and equal for any ix < 2^32
    const float fx = (float)(uint32_t)ix, fy = (float)(uint32_t)iy;
    float x = P.n_mod[0] + P.u_mod[0] * fx + P.v_mod[0] * fy;
    float y = P.n_mod[1] + P.u_mod[1] * fx + P.v_mod[1] * fy;
    float z = P.n_mod[2] + P.u_mod[2] * fx + P.v_mod[2] * fy;
    const float r = kR ? rn : rsqrt21(x, y, z);
    rn = r;
    rmd[0] = x * r; rmd[1] = y * r; rmd[2] = z * r;
}
__device__ __forceinline__ void primary_ray(const TraceParams& P, int32_t ix, int32_t iy, float rmd[3]) {
    float rn;
    primary_ray<false>(P, ix, iy, rmd, rn);
}

__device__ __forceinline__ void wave_count_add(unsigned long long* dst, uint32_t v) {
    // counting builds only; the compiler's atomic optimizer folds the active
    // lanes of a wave into one atomic (lanes of edge tiles may have exited)
    if (v) atomicAdd(dst, (unsigned long long)v);
}

// ------------------------------------------------------------- KD trace v2

// Issues the four dwordx4 loads of a 64-B record together and consumes them
// before any branch, so a visit costs one memory round trip (left to itself
// hipcc sinks the conditionally used loads into the branches: three
// dependent round trips per visit).
__device__ __forceinline__ void load_record(const float4* __restrict__ p, float4& r0, float4& r1,
                                            float4& r2, float4& r3) {
    r0 = p[0]; r1 = p[1]; r2 = p[2]; r3 = p[3];
    asm volatile("" ::"v"(r0.x), "v"(r0.y), "v"(r0.z), "v"(r0.w), "v"(r1.x), "v"(r1.y), "v"(r1.z),
                 "v"(r1.w), "v"(r2.x), "v"(r2.y), "v"(r2.z), "v"(r2.w), "v"(r3.x), "v"(r3.y), "v"(r3.z),
                 "v"(r3.w));
}

// s1 (the left child's high bound) and s2 (the right child's low bound) on
// the cut axis, from an interior record's boxes (k_cam_nodes).
__device__ __forceinline__ float rec_s1(float4 r0, float4 r1, uint32_t axis) {
    return axis == 0 ? r0.y : axis == 1 ? r0.w : r1.y;
}
__device__ __forceinline__ float rec_s2(float4 r1, float4 r2, uint32_t axis) {
    return axis == 0 ? r1.z : axis == 1 ? r2.x : r2.z;
}

struct Ray {
    float rx, ry, rz;          // object-space direction, TD/Trixel.cu:64-66
    float odx, ody, odz;       // object translation, TD/Trixel.cu:60-62
    float ix, iy, iz;          // 1 / r
    float ox, oy, oz;          // od / r
    bool sx, sy, sz;           // r > 0
};

typedef float f2v __attribute__((ext_vector_type(2)));

// Slab parameters of one node, TD/Trixel.cu:76-95: entry maxt0, exit mint1.
__device__ __forceinline__ void slab_vals(const Ray& R, float lx, float hx, float ly, float hy, float lz,
                                          float hz, float& maxt0, float& mint1) {
    const float t0x = R.sx ? lx * R.ix : hx * R.ix;
    const float t1x = R.sx ? hx * R.ix : lx * R.ix;
    const float t0y = R.sy ? ly * R.iy : hy * R.iy;
    const float t1y = R.sy ? hy * R.iy : ly * R.iy;
    const float t0z = R.sz ? lz * R.iz : hz * R.iz;
    const float t1z = R.sz ? hz * R.iz : lz * R.iz;
    maxt0 = fmaxf(t0z + R.oz, fmaxf(t0x + R.ox, t0y + R.oy));
    mint1 = fminf(t1z + R.oz, fminf(t1x + R.ox, t1y + R.oy));
}

// The same for a kFast walk (untranslated, every ray component normal and
// nonzero, ordered boxes): each od/r term is a signed zero (0/r), and adding
// it changes at most the sign of a zero t, which no comparison downstream
// tells apart (the entry test, the split-plane order, the products t * dir),
// so it is skipped; with 1/r finite and nonzero and lo <= hi, the product of
// lo is the smaller one exactly when r > 0, so min / max of an axis's two
// products are the reference's sign-selected t0 / t1.  Each axis's two
// products are one v_pk_mul_f32 (each half rounds as the scalar multiply
// does) of the record's (lo, hi) pair by the broadcast 1/r.
__device__ __forceinline__ void slab_fast(f2v bx, f2v by, f2v bz, float ix, float iy, float iz, float& maxt0,
                                          float& mint1) {
    const f2v px = bx * ix, py = by * iy, pz = bz * iz;
    maxt0 = fmaxf(fminf(pz.x, pz.y), fmaxf(fminf(px.x, px.y), fminf(py.x, py.y)));
    mint1 = fminf(fmaxf(pz.x, pz.y), fminf(fmaxf(px.x, px.y), fmaxf(py.x, py.y)));
}

// slab_fast for both child boxes of a record (r0..r2: the left box's (lo,
// hi) pairs on x, y, z, then the right box's), for a walk whose live rays all
// lie in one octant (kOct bit k: component k positive; 8: any).  Then the
// reference's sign-selected t0 of an axis (TD/Trixel.cu:76-83) is the product
// of lo (r > 0) or of hi (r < 0), known at compile time, and each box takes
// one max3 and one min3 after its products instead of a min and a max per
// axis (the same values: with lo <= hi and 1/r of the component's sign, the
// selected product is the smaller one).  pool_walk_oct instantiates the walk
// per octant, so no per-slot switch is paid.
#ifndef RT_OCT_WALKS
#define RT_OCT_WALKS 1
#endif
template <int kOct>
__device__ __forceinline__ void slab_pair_oct(float4 r0, float4 r1, float4 r2, float ix, float iy, float iz,
                                              float& lt0, float& lt1, float& rt0, float& rt1) {
    if constexpr (kOct >= 8) {
        slab_fast(f2v{r0.x, r0.y}, f2v{r0.z, r0.w}, f2v{r1.x, r1.y}, ix, iy, iz, lt0, lt1);
        slab_fast(f2v{r1.z, r1.w}, f2v{r2.x, r2.y}, f2v{r2.z, r2.w}, ix, iy, iz, rt0, rt1);
    } else {
        const f2v ax = f2v{r0.x, r0.y} * ix, ay = f2v{r0.z, r0.w} * iy, az = f2v{r1.x, r1.y} * iz;
        const f2v bx = f2v{r1.z, r1.w} * ix, by = f2v{r2.x, r2.y} * iy, bz = f2v{r2.z, r2.w} * iz;
        constexpr bool sx = (kOct & 1) != 0, sy = (kOct & 2) != 0, sz = (kOct & 4) != 0;
        lt0 = fmaxf(sz ? az.x : az.y, fmaxf(sx ? ax.x : ax.y, sy ? ay.x : ay.y));
        lt1 = fminf(sz ? az.y : az.x, fminf(sx ? ax.y : ax.x, sy ? ay.y : ay.x));
        rt0 = fmaxf(sz ? bz.x : bz.y, fmaxf(sx ? bx.x : bx.y, sy ? by.x : by.y));
        rt1 = fminf(sz ? bz.y : bz.x, fminf(sx ? bx.y : bx.x, sy ? by.y : by.x));
    }
}

// slab_pair_oct for translated walks (round 6): the reference's t = b * (1/r)
// + od/r per axis (TD/Trixel.cu:76-95), the product of the near bound (lo for
// r > 0) plus the offset for t0 and of the far bound for t1 -- with the
// octant known at compile time the selection is fixed; for mixed octants
// (kOct 8) min / max of the two products select it (lo <= hi, 1/r of the
// component's sign).  Products as v_pk_mul_f32 pairs, then the offsets.
template <int kOct>
__device__ __forceinline__ void slab_pair_xoct(float4 r0, float4 r1, float4 r2, float ix, float iy, float iz, float ox,
                                               float oy, float oz, float& lt0, float& lt1, float& rt0, float& rt1) {
    const f2v ax = f2v{r0.x, r0.y} * ix, ay = f2v{r0.z, r0.w} * iy, az = f2v{r1.x, r1.y} * iz;
    const f2v bx = f2v{r1.z, r1.w} * ix, by = f2v{r2.x, r2.y} * iy, bz = f2v{r2.z, r2.w} * iz;
    float anx, afx, any, afy, anz, afz, bnx, bfx, bny, bfy, bnz, bfz;
    if constexpr (kOct >= 8) {
        anx = fminf(ax.x, ax.y); afx = fmaxf(ax.x, ax.y);
        any = fminf(ay.x, ay.y); afy = fmaxf(ay.x, ay.y);
        anz = fminf(az.x, az.y); afz = fmaxf(az.x, az.y);
        bnx = fminf(bx.x, bx.y); bfx = fmaxf(bx.x, bx.y);
        bny = fminf(by.x, by.y); bfy = fmaxf(by.x, by.y);
        bnz = fminf(bz.x, bz.y); bfz = fmaxf(bz.x, bz.y);
    } else {
        constexpr bool sx = (kOct & 1) != 0, sy = (kOct & 2) != 0, sz = (kOct & 4) != 0;
        anx = sx ? ax.x : ax.y; afx = sx ? ax.y : ax.x;
        any = sy ? ay.x : ay.y; afy = sy ? ay.y : ay.x;
        anz = sz ? az.x : az.y; afz = sz ? az.y : az.x;
        bnx = sx ? bx.x : bx.y; bfx = sx ? bx.y : bx.x;
        bny = sy ? by.x : by.y; bfy = sy ? by.y : by.x;
        bnz = sz ? bz.x : bz.y; bfz = sz ? bz.y : bz.x;
    }
    const f2v o2 = f2v{ox, oy};
    const f2v la = f2v{anx, any} + o2, lb = f2v{afx, afy} + o2, ra = f2v{bnx, bny} + o2, rb = f2v{bfx, bfy} + o2;
    lt0 = fmaxf(anz + oz, fmaxf(la.x, la.y));
    lt1 = fminf(afz + oz, fminf(lb.x, lb.y));
    rt0 = fmaxf(bnz + oz, fmaxf(ra.x, ra.y));
    rt1 = fminf(bfz + oz, fminf(rb.x, rb.y));
}

// Slab test of one node, TD/Trixel.cu:76-95,146: entry/exit parameters and
// whether the reference descends into the node.
__device__ __forceinline__ bool slab(const Ray& R, float lx, float hx, float ly, float hy, float lz,
                                     float hz, float& maxt0, float& mint1) {
    slab_vals(R, lx, hx, ly, hy, lz, hz, maxt0, mint1);
    return pred::enter(maxt0, mint1);
}

// Moller-Trumbore at a leaf, TD/Trixel.cu:98-145; updates (d, best) on a
// strictly nearer accepted hit.
__device__ __forceinline__ bool leaf_test_rec(const Ray& R, const float4 A, const float4 B, const float4 Cq,
                                              uint32_t t, float& d, uint32_t& best) {
    const float e1x = A.x, e1y = A.y, e1z = A.z;
    const float e2x = A.w, e2y = B.x, e2z = B.y;
    const float dtx = B.z, dty = B.w, dtz = Cq.x;
    float qpx, qpy, qpz;
    cross3(qpx, qpy, qpz, R.rx, R.ry, R.rz, e2x, e2y, e2z);
    const float f = dot3(qpx, qpy, qpz, e1x, e1y, e1z);
    if (!(f < kEpsF && f > -kEpsF)) {
        const float pe1 = 1.0f / f;   // == (float)(1.0 / (double)f)
        const float tx = dtx - R.odx, ty = dty - R.ody, tz = dtz - R.odz;
        const float u = pe1 * dot3(qpx, qpy, qpz, tx, ty, tz);
        float qx, qy, qz;
        cross3(qx, qy, qz, tx, ty, tz, e1x, e1y, e1z);
        const float v = pe1 * dot3(R.rx, R.ry, R.rz, qx, qy, qz);
        const float w = pe1 * dot3(e2x, e2y, e2z, qx, qy, qz);
        // (u+v) > 1 + 1e-16 is (u+v) > 1.0 in double
        if ((w < d) && !((u < kEpsF) || (v < kEpsF) || ((u + v) > 1.0f) || (w < kEpsF))) {
            d = w;
            best = t;
            return true;
        }
    }
    return false;
}

// leaf_test_rec for a ray from the camera (no object translation): t = d_t,
// so cross(t, e1) is the record's d_q and dot(e2, cross(t, e1)) its d_w,
// both computed by k_cam_tri with the same float operations (products
// commute exactly): 14 fewer VALU operations per leaf visit, the same bits.
// Every lane evaluates the whole test and selects (no exec-mask branches;
// the 1/f of a rejected f is never used).
__device__ __forceinline__ bool leaf_test_cam(const Ray& R, const float4 A, const float4 B, const float4 Cq,
                                              const float4 Dq, uint32_t t, float& d, uint32_t& best) {
    const float e1x = A.x, e1y = A.y, e1z = A.z;
    const float e2x = A.w, e2y = B.x, e2z = B.y;
    const float tx = B.z, ty = B.w, tz = Cq.x;
    float qpx, qpy, qpz;
    cross3(qpx, qpy, qpz, R.rx, R.ry, R.rz, e2x, e2y, e2z);
    const float f = dot3(qpx, qpy, qpz, e1x, e1y, e1z);
    // pe1 == (float)(1.0 / (double)f): rcp_nr unless a lane's |f| is 2^126 or
    // more (|f| below 2^-126 is below 1e-16, rejected whatever pe1 is)
    const float pe1 = __ballot(fabsf(f) >= 0x1p126f) == 0ull ? rcp_nr(f) : 1.0f / f;
    const float u = pe1 * dot3(qpx, qpy, qpz, tx, ty, tz);
    const float v = pe1 * dot3(R.rx, R.ry, R.rz, Cq.y, Cq.z, Cq.w);
    const float w = pe1 * Dq.x;
    const bool acc = !(f < kEpsF && f > -kEpsF) & (w < d) &
                     !((u < kEpsF) | (v < kEpsF) | ((u + v) > 1.0f) | (w < kEpsF));
    d = acc ? w : d;
    best = acc ? t : best;
    return acc;
}

// leaf_test_rec for the translated kFast walks (round 6: object transforms
// with an offset, and the shadow rays from the light): the same float
// expressions, every term computed and selected (no exec-mask branches), and
// pe1 from rcp_nr as in leaf_test_cam.
__device__ __forceinline__ bool leaf_test_xf(const Ray& R, const float4 A, const float4 B, const float4 Cq, uint32_t t,
                                             float& d, uint32_t& best) {
    const float e1x = A.x, e1y = A.y, e1z = A.z;
    const float e2x = A.w, e2y = B.x, e2z = B.y;
    const float dtx = B.z, dty = B.w, dtz = Cq.x;
    float qpx, qpy, qpz;
    cross3(qpx, qpy, qpz, R.rx, R.ry, R.rz, e2x, e2y, e2z);
    const float f = dot3(qpx, qpy, qpz, e1x, e1y, e1z);
    const float pe1 = __ballot(fabsf(f) >= 0x1p126f) == 0ull ? rcp_nr(f) : 1.0f / f;
    const float tx = dtx - R.odx, ty = dty - R.ody, tz = dtz - R.odz;
    const float u = pe1 * dot3(qpx, qpy, qpz, tx, ty, tz);
    float qx, qy, qz;
    cross3(qx, qy, qz, tx, ty, tz, e1x, e1y, e1z);
    const float v = pe1 * dot3(R.rx, R.ry, R.rz, qx, qy, qz);
    const float w = pe1 * dot3(e2x, e2y, e2z, qx, qy, qz);
    const bool acc = !(f < kEpsF && f > -kEpsF) & (w < d) &
                     !((u < kEpsF) | (v < kEpsF) | ((u + v) > 1.0f) | (w < kEpsF));
    d = acc ? w : d;
    best = acc ? t : best;
    return acc;
}

__device__ __forceinline__ bool leaf_test(const Ray& R, const float4* __restrict__ trec, uint32_t t,
                                          float& d, uint32_t& best) {
    return leaf_test_rec(R, trec[4 * (size_t)t], trec[4 * (size_t)t + 1], trec[4 * (size_t)t + 2], t, d, best);
}

// intersect_voxel_cuda (TD/Trixel.cu:41-172) fused with set_cam_cuda +
// color_cam_cuda (TD/Camera.cu:12-69), v2 layout.  A node's record carries its
// children's boxes, so a child's slab test runs when the parent decides to
// push it: children that the reference would pop and reject are never
// fetched, the deferred sibling keeps its (maxt0, mint1) in LDS, and every
// effectful visit happens in the reference's DFS order.
template <bool kTranslated, bool kWriteHit, bool kCount>
__global__ __launch_bounds__(kTileWKd * kTileH) void k_trace_kd2(TraceParams P) {
    constexpr int kB = kTileWKd * kTileH;
    __shared__ uint32_t s_ref[kMaxDepth * kB];
    __shared__ float s_t0[kMaxDepth * kB];
    __shared__ float s_t1[kMaxDepth * kB];
    Pixel px;
    if (!pixel_of_thread(P, px)) return;  // no barriers in this kernel
    const unsigned long long t_start = P.dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;

    float cam[3];
    primary_ray(P, px.x, px.y, cam);
    const float* X = P.xf;
    Ray R;
    R.odx = X[3]; R.ody = X[7]; R.odz = X[11];
    R.rx = -1 * (X[0] * -cam[0] + X[1] * -cam[1] + X[2] * -cam[2]);
    R.ry = -1 * (X[4] * -cam[0] + X[5] * -cam[1] + X[6] * -cam[2]);
    R.rz = -1 * (X[8] * -cam[0] + X[9] * -cam[1] + X[10] * -cam[2]);
    R.ix = 1 / R.rx; R.iy = 1 / R.ry; R.iz = 1 / R.rz;
    R.ox = R.odx / R.rx; R.oy = R.ody / R.ry; R.oz = R.odz / R.rz;
    R.sx = R.rx > 0; R.sy = R.ry > 0; R.sz = R.rz > 0;
    // dir and ds for each one-hot cut axis (TD/Trixel.cu:88-90)
    const float dir_a[3] = {(R.rx * 1.0f) + (R.ry * 0.0f) + (R.rz * 0.0f),
                            (R.rx * 0.0f) + (R.ry * 1.0f) + (R.rz * 0.0f),
                            (R.rx * 0.0f) + (R.ry * 0.0f) + (R.rz * 1.0f)};
    const float ds_a[3] = {(R.odx * 1.0f) + (R.ody * 0.0f) + (R.odz * 0.0f),
                           (R.odx * 0.0f) + (R.ody * 1.0f) + (R.odz * 0.0f),
                           (R.odx * 0.0f) + (R.ody * 0.0f) + (R.odz * 1.0f)};

    float d = kDrawDistance;
    uint32_t best = kMiss;
    uint32_t n_int = 0, n_leaf = 0, n_acc = 0, n_desc = 0;
    const int lane_col = (int)threadIdx.x;
    int sp = 0;
    uint32_t ref = P.root_ref;
    float cmax = 0.0f, cmin = 0.0f;
    bool have = true;
    if (!(ref & kLeafBit)) {
        if (kCount) n_int++;
        have = slab(R, P.root_box[0], P.root_box[1], P.root_box[2], P.root_box[3], P.root_box[4],
                    P.root_box[5], cmax, cmin);
        if (kCount && have) n_desc++;
    }
    if (P.debug & 1) have = false;
    uint32_t n_visit = 0;
    while (have) {
        if (P.dbg) n_visit++;
        if (ref & kLeafBit) {
            if (kCount) n_leaf++;
            const bool acc = leaf_test(R, P.trec, ref & ~kLeafBit, d, best);
            if (kCount && acc) n_acc++;
        } else {
            float4 r0, r1, r2, r3;
            load_record(P.inode + 4 * (size_t)ref, r0, r1, r2, r3);
            const uint32_t lw = __float_as_uint(r3.z);
            const uint32_t axis = (lw >> kAxisShift) & 3u;
            const uint32_t L = lw & ~(3u << kAxisShift), Rr = __float_as_uint(r3.w) & ~kTinyS1Bit;
            const float dir = axis == 0 ? dir_a[0] : axis == 1 ? dir_a[1] : dir_a[2];
            const float mx = cmax * dir, mn = cmin * dir;
            float s1;
            bool lt, gt;  // the reference's double tests against s2 (TD/Trixel.cu:155-157)
            if (kTranslated) {
                const float ds = axis == 0 ? ds_a[0] : axis == 1 ? ds_a[1] : ds_a[2];
                s1 = (float)((double)rec_s1(r0, r1, axis) + kEps + (double)ds);
                const float s2 = rec_s2(r1, r2, axis) + ds;
                lt = pred::lt_eps(mx, s2);
                gt = pred::gt_eps(mn, s2);
            } else {  // ds == 0: the record's exact float thresholds
                s1 = pred::add_eps(rec_s1(r0, r1, axis));
                lt = mx < r3.y;
                gt = mn > r3.x;
            }
            // Push order of TD/Trixel.cu:155-168.  `first` is popped next,
            // `second` (if pushed) after first's subtree.
            bool left_first, push_second;
            if (lt) {
                left_first = true;
                push_second = gt;
            } else {
                left_first = false;
                push_second = (mn < s1 || mx < s1);
            }
            const uint32_t first = left_first ? L : Rr;
            const uint32_t second = left_first ? Rr : L;
            // slab tests of the children that would be popped (boxes in r0..r2)
            float f0 = 0.0f, f1 = 0.0f, g0 = 0.0f, g1 = 0.0f;
            bool keep_first = true, keep_second = push_second;
            if (!(first & kLeafBit)) {
                if (kCount) n_int++;
                keep_first = left_first ? slab(R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, f0, f1)
                                        : slab(R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w, f0, f1);
                if (kCount && keep_first) n_desc++;
            }
            if (push_second && !(second & kLeafBit)) {
                if (kCount) n_int++;
                keep_second = left_first ? slab(R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w, g0, g1)
                                         : slab(R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, g0, g1);
                if (kCount && keep_second) n_desc++;
            }
            if (keep_first) {
                if (keep_second) {
                    if (sp >= P.max_depth) { atomicOr(P.err, 1); break; }
                    const int k = sp * kB + lane_col;
                    s_ref[k] = second; s_t0[k] = g0; s_t1[k] = g1;
                    sp++;
                }
                ref = first; cmax = f0; cmin = f1;
                continue;
            }
            if (keep_second) {
                ref = second; cmax = g0; cmin = g1;
                continue;
            }
        }
        if (sp == 0) break;
        sp--;
        const int k = sp * kB + lane_col;
        ref = s_ref[k]; cmax = s_t0[k]; cmin = s_t1[k];
    }

    uint32_t argb = kBackground;
    if (best != kMiss) {
        // nearest-hit writes of TD/Trixel.cu:128-140, done once for the final hit
        const float4 N = P.shade[2 * (size_t)best];
        const float4 M = P.shade[2 * (size_t)best + 1];
        const float pnt[3] = {d * R.rx + R.odx, d * R.ry + R.ody, d * R.rz + R.odz};
        // norm.device_rotate(rot_m, i, -1), TD/vector.cuh:23-33
        const float ax = -1 * N.x, ay = -1 * N.y, az = -1 * N.z;
        const float nrm[3] = {(ax * X[0] + ay * X[1] + az * X[2]) * -1,
                              (ax * X[4] + ay * X[5] + az * X[6]) * -1,
                              (ax * X[8] + ay * X[9] + az * X[10]) * -1};
        const float rad[3] = {M.x, M.y, M.z};
        argb = phong(pnt, nrm, cam, rad);
    }
    put_pixel(P, px.out, argb, best != kMiss);
    if (kWriteHit) P.hit[px.out] = best == kMiss ? (int64_t)-1 : (int64_t)best;
    if (kCount) {
        wave_count_add(&P.counters[0], n_int);
        wave_count_add(&P.counters[1], n_leaf);
        wave_count_add(&P.counters[2], n_acc);
        wave_count_add(&P.counters[3], best != kMiss ? 1u : 0u);
        wave_count_add(&P.counters[4], n_desc);
    }
    if (P.dbg) {  // diagnostic build: wave start/end clock and its max visits
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        const size_t wv = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        atomicMax(&P.dbg[3 * wv + 2], (unsigned long long)n_visit);
        if (((int)threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)threadIdx.x & 63)) {
            P.dbg[3 * wv] = t_start;
            P.dbg[3 * wv + 1] = t_end;
        }
    }
}

// ------------------------------------------------------------- KD trace v3

// Wave-cooperative traversal.  With no early termination the SET of nodes a
// ray visits does not depend on the order of the visits, and the reference's
// result is the accepted candidate with the smallest w, ties going to the one
// its DFS visits first (strict `w < d`, TD/Trixel.cu:127).  So a wave pools
// the (ray, node) work items of its 64 rays in one LDS stack and every lane
// takes an item per iteration, whatever ray it belongs to: the wave runs
// ~sum(visits)/64 iterations instead of max(visits).  Each item carries its
// DFS path code (bit = "second child popped" at each level), so the
// lexicographic minimum of (w, code left-aligned) -- one 64-bit LDS atomic
// min per candidate -- is exactly the reference's winner.
//
// The path code is stored with a leading marker bit: the root is 1, a node
// with code m has children 2m (popped first) and 2m + 1, so its depth is the
// position of the marker and any tree the LDS stack admits (height <=
// kMaxDepth = 24: 25 bits) fits beside the 6-bit ray index.
constexpr int kPoolCap = kPoolCapMax;
constexpr int kCodeBits = kMaxDepth;       // left-aligned code width in the key
constexpr uint32_t kCodeMarkMask = (1u << 26) - 1;

// Both records of an iteration are issued before either is consumed, and a
// scheduling barrier after the loads lets item 0 wait only for its own record
// (vmcnt counts loads in order) while item 1's is still in flight (round 2:
// an empty asm reading all 32 registers made the wave wait for both; dragon
// 1080p 14.6k -> 15.3k FPS, solo 86.7 -> 82.2 us).
#define RT_RECORD_FENCE() __builtin_amdgcn_sched_barrier(0)

struct Item {
    uint32_t ref;      // node ref (kLeafBit | tri, or interior index)
    float t0, t1;      // the node's (maxt0, mint1) for interior refs
    uint32_t meta;     // ray << 26 | marked path code
};

// The key bits of a marked path code: the code left-aligned in kCodeBits.
__device__ __forceinline__ uint32_t code_key(uint32_t marked) {
    const uint32_t depth = 31u - (uint32_t)__builtin_clz(marked);
    return (marked ^ (1u << depth)) << (kCodeBits - depth);
}

// Pool capacity per wave for kRays rays (the DFS fallback keeps any
// capacity >= 89 correct; these cover the measured peaks with margin).
#ifndef RT_POOL_CAP_R32
#define RT_POOL_CAP_R32 448
#endif
#ifndef RT_POOL_CAP_R16
#define RT_POOL_CAP_R16 352
#endif
// 8 rays: 448 items (30.6 KB per 4-wave block, 5 blocks per CU).  Two
// frames in flight (r02): 960x540 27.4k FPS at 512 (34.7 KB, 4 blocks),
// 31.2k at 448, 33.1k at 384; a rank of 4 at 1080p 36.7 / 32.8 / 31.1 us, of
// 8 24.1 / 24.2 / 25.9 us: 448 loses nowhere.
#ifndef RT_POOL_CAP_R8
#define RT_POOL_CAP_R8 448
#endif
template <int kRays>
constexpr int pool_cap_for() {
    return kRays == 32 ? RT_POOL_CAP_R32 : kRays == 16 ? RT_POOL_CAP_R16 : RT_POOL_CAP_R8;
}

// Per-ray data of the pool walk in LDS: rd[0] = (rx, ry, rz, 1/rx),
// rd[1] = (1/ry, 1/rz, odx/rx, ody/ry), rd[2] = (odz/rz, dir per cut axis),
// translated walks add rd[3] = (od, ds of axis 0), rd[4] = (ds of axes 1-2,
// shadow walks: Lmax, hit triangle).
// Per-ray data of the pool walk in a wave's LDS: six float2 fields per ray
// (ten for translated and shadow walks), field-major -- field k of ray r at
// ray[k * stride + r], stride kRays (48 for 32 rays, RayLayout) -- so that
// every read of a field by the lanes of a wave
// (items of up to kRays distinct rays) hits distinct banks, whatever width
// the compiler reads it with: for kRays <= 16 a ds_read_b64 (64 banks) and a
// ds_read_b32 / ds_read2_b32 (32 banks) of one component both spread the
// rays over distinct banks.  Round 2's ray-major float4 records (48 B per
// ray) put rays r and r + 8 on the same banks: 1.36 conflict cycles per LDS
// instruction in the 16-ray instance at C4 (the 8-ray one 0.05); float4
// fields (r03a) still conflicted through the ds_read2_b32 halves the compiler
// split them into (0.71).
//   f0 (rx, ry)  f1 (rz, 1/rx)  f2 (1/ry, 1/rz)  f3 (odx/rx, ody/ry)
//   f4 (odz/rz, dir axis 0)  f5 (dir axis 1, dir axis 2)
//   translated / shadow walks add f6 (odx, ody)  f7 (odz, ds axis 0)
//   f8 (ds axis 1, ds axis 2)  f9 (Lmax, hit triangle)
// The 32-ray instance (multi-frame launches of small frames, auto_rays)
// spaces its fields 48 float2s apart, so that two fields of one ray read
// together do not share banks: C3 65.6-65.7k -> 66.9-67.0k FPS, knot
// 960x540 37.1k -> 37.7k (r04va; 40 gave the same).
#ifndef RT_RAY_STRIDE32
#define RT_RAY_STRIDE32 48
#endif
template <int kRays>
struct RayLayout {
    static constexpr int kStride = kRays == 32 ? RT_RAY_STRIDE32 : kRays;  // float2s between the fields of one ray
};

__device__ __forceinline__ void store_ray(float2* rd, int stride, const Ray& R, bool translated, float lmax,
                                          uint32_t self) {
    // dir and ds for each one-hot cut axis (TD/Trixel.cu:88-90)
    const float d0 = (R.rx * 1.0f) + (R.ry * 0.0f) + (R.rz * 0.0f);
    const float d1 = (R.rx * 0.0f) + (R.ry * 1.0f) + (R.rz * 0.0f);
    const float d2 = (R.rx * 0.0f) + (R.ry * 0.0f) + (R.rz * 1.0f);
    rd[0] = make_float2(R.rx, R.ry);
    rd[stride] = make_float2(R.rz, R.ix);
    rd[2 * stride] = make_float2(R.iy, R.iz);
    rd[3 * stride] = make_float2(R.ox, R.oy);
    rd[4 * stride] = make_float2(R.oz, d0);
    rd[5 * stride] = make_float2(d1, d2);
    if (translated) {
        const float e0 = (R.odx * 1.0f) + (R.ody * 0.0f) + (R.odz * 0.0f);
        const float e1 = (R.odx * 0.0f) + (R.ody * 1.0f) + (R.odz * 0.0f);
        const float e2 = (R.odx * 0.0f) + (R.ody * 0.0f) + (R.odz * 1.0f);
        rd[6 * stride] = make_float2(R.odx, R.ody);
        rd[7 * stride] = make_float2(R.odz, e0);
        rd[8 * stride] = make_float2(e1, e2);
        rd[9 * stride] = make_float2(lmax, __uint_as_float(self));
    }
}

// Derived fields of a ray whose direction and translation are set.
// kPlain: an untranslated instance, whose od components are signed zeros:
// od / r is then a signed zero of sign(od) ^ sign(r), or NaN when r is 0 or
// NaN (0 / 0), computed without a division; 1 / r takes rcp_nr when every
// lane's components are in its range.
__device__ __forceinline__ float zero_over(float od, float r) {
    return (r == 0.0f || r != r) ? __builtin_nanf("")
                                 : __uint_as_float((__float_as_uint(od) ^ __float_as_uint(r)) & 0x80000000u);
}
template <bool kPlain = false>
__device__ __forceinline__ void finish_ray(Ray& R) {
    if (kPlain && __ballot(!(rcp_nr_ok(R.rx) && rcp_nr_ok(R.ry) && rcp_nr_ok(R.rz))) == 0ull) {
        R.ix = rcp_nr(R.rx); R.iy = rcp_nr(R.ry); R.iz = rcp_nr(R.rz);
    } else {
        R.ix = 1 / R.rx; R.iy = 1 / R.ry; R.iz = 1 / R.rz;
    }
    if (kPlain) {
        R.ox = zero_over(R.odx, R.rx); R.oy = zero_over(R.ody, R.ry); R.oz = zero_over(R.odz, R.rz);
    } else {
        R.ox = R.odx / R.rx; R.oy = R.ody / R.ry; R.oz = R.odz / R.rz;
    }
    R.sx = R.rx > 0; R.sy = R.ry > 0; R.sz = R.rz > 0;
}

// The primary ray of a pixel (TD/Camera.cu:103-104) and its object-space form
// (TD/Trixel.cu:60-66); dead lanes get a harmless +z ray.
// kR / rn: as primary_ray's (a live lane's normalisation factor, given or returned).
template <bool kR = false, bool kPlain = false>
__device__ __forceinline__ void camera_ray(const TraceParams& P, const Pixel& px, bool live, float cam[3], Ray& R,
                                           float& rn) {
    cam[0] = 0.0f; cam[1] = 0.0f; cam[2] = 1.0f;
    if (live) primary_ray<kR>(P, px.x, px.y, cam, rn);
    const float* X = P.xf;
    R.odx = X[3]; R.ody = X[7]; R.odz = X[11];
    R.rx = -1 * (X[0] * -cam[0] + X[1] * -cam[1] + X[2] * -cam[2]);
    R.ry = -1 * (X[4] * -cam[0] + X[5] * -cam[1] + X[6] * -cam[2]);
    R.rz = -1 * (X[8] * -cam[0] + X[9] * -cam[1] + X[10] * -cam[2]);
    finish_ray<kPlain>(R);
}
__device__ __forceinline__ void camera_ray(const TraceParams& P, const Pixel& px, bool live, float cam[3], Ray& R) {
    float rn = 1.0f;
    camera_ray<false>(P, px, live, cam, R, rn);
}

// Shadow walks on the segment (round 6): 0 follows the whole ray beyond the
// hit, as rounds 1-5 did (the same images; A/B builds only -- the oracle's
// counters are the segment walk's).
#ifndef RT_SHADOW_SEGMENT
#define RT_SHADOW_SEGMENT 1
#endif
// The reference's root visit (TD/Trixel.cu:53,71-95): a leaf root is always
// visited, an interior root when its slab test passes.  kSeg: a shadow
// segment's walk, which enters a box only where the segment does (its entry
// parameter below Lmax = lim, round 6; oracle.c trace_shadow).
template <bool kCount, bool kSeg = false>
__device__ __forceinline__ bool root_pass(const TraceParams& P, const Ray& R, bool live, float& t0, float& t1,
                                          uint32_t& n_int, uint32_t& n_desc, float lim = 0.0f) {
    bool has = false;
    t0 = 0.0f; t1 = 0.0f;
    if (live) {
        if (P.root_ref & kLeafBit) {
            has = true;
        } else {
            if (kCount) n_int++;
            has = slab(R, P.root_box[0], P.root_box[1], P.root_box[2], P.root_box[3], P.root_box[4],
                       P.root_box[5], t0, t1);
            if (kSeg && RT_SHADOW_SEGMENT) has = has && t0 < lim;
            if (kCount && has) n_desc++;
        }
    }
    if (P.debug & 1) has = false;
    return has;
}

// Seeds the pool with the root item of every lane whose root test passes (or
// a leaf root); returns the item count.
template <bool kCount, bool kSeg = false>
__device__ __forceinline__ int seed_root(const TraceParams& P, uint4* items, const Ray& R, bool live, int lane,
                                         uint32_t& n_int, uint32_t& n_desc, float lim = 0.0f) {
    float r0t0, r0t1;
    const bool has = root_pass<kCount, kSeg>(P, R, live, r0t0, r0t1, n_int, n_desc, lim);
    const unsigned long long b = __ballot(has);
    const uint32_t off = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    if (has) items[off] = make_uint4(P.root_ref, __float_as_uint(r0t0), __float_as_uint(r0t1), ((uint32_t)lane << 26) | 1u);
    __builtin_amdgcn_wave_barrier();
    return __builtin_popcountll(b);
}

// One popped item's outcome: up to two children and a candidate hit.
struct Visit {
    uint4 ca, cb;      // the first and second child items (TD/Trixel.cu:155-168 order)
    bool ka, kb;       // whether each is pushed
    bool cand;
    unsigned long long key;
    uint32_t ctri;
};

// The 64-B record of an item: a node's child-box record, or a leaf's
// triangle record (tri_world relative to the camera).
__device__ __forceinline__ const float4* record_of(const TraceParams& P, uint32_t ref) {
    return (ref & kLeafBit) ? P.trec + 4 * (size_t)(ref & ~kLeafBit) : P.inode + 4 * (size_t)ref;
}

// record_of for kFast walks: the records are one allocation (inode, then
// trec at byte offset P.leaf_off < 4 GiB), so the address is P.inode plus a
// 32-bit offset: ref << 6 drops the leaf bit, and a leaf adds leaf_off.
__device__ __forceinline__ const float4* record_fast(const TraceParams& P, uint32_t ref) {
    const uint32_t off = (ref << 6) + ((int32_t)ref < 0 ? P.leaf_off : 0u);
    return (const float4*)((const char*)P.inode + off);
}

// The per-ray data of an item's ray from LDS (see store_ray), as the float4s
// (q2 = (odz/rz, dir per axis), q3 = (od, ds axis 0), q4 = (ds axes 1-2,
// Lmax, hit triangle)) the visits read.
// kFast walks read the first three fields only (direction and 1/r: no
// offsets, and the direction per cut axis is the component itself).
// kOdP (round 6): a translated nearest-hit walk whose LDS holds six fields
// only -- the offset od and ds per cut axis (r_a * 1 + r_b * 0 + r_c * 0 of
// od: od's component, up to the sign of a zero, which no compare sees) are
// the transform's own, uniform over the wave (xf = P.xf).
template <bool kTranslated, int kStride, bool kFast = false, bool kOdP = false>
__device__ __forceinline__ void ray_of(const float2* rd, Ray& Q, float4& q2, float4& q3, float4& q4,
                                       const float* xf = nullptr) {
    const float2 z = make_float2(0.0f, 0.0f);
    const float2 f0 = rd[0], f1 = rd[kStride], f2 = rd[2 * kStride];
    const float2 f3 = kFast ? z : rd[3 * kStride], f4 = kFast ? z : rd[4 * kStride], f5 = kFast ? z : rd[5 * kStride];
    const float2 f6 = kTranslated ? (kOdP ? make_float2(xf[3], xf[7]) : rd[6 * kStride]) : z;
    const float2 f7 = kTranslated ? (kOdP ? make_float2(xf[11], xf[3]) : rd[7 * kStride]) : z;
    const float2 f8 = kTranslated ? (kOdP ? make_float2(xf[7], xf[11]) : rd[8 * kStride]) : z;
    const float2 f9 = kTranslated && !kOdP ? rd[9 * kStride] : z;
    q2 = make_float4(f4.x, f4.y, f5.x, f5.y);
    q3 = make_float4(f6.x, f6.y, f7.x, f7.y);
    q4 = make_float4(f8.x, f8.y, f9.x, f9.y);
    Q.rx = f0.x; Q.ry = f0.y; Q.rz = f1.x; Q.ix = f1.y;
    Q.iy = f2.x; Q.iz = f2.y; Q.ox = f3.x; Q.oy = f3.y;
    Q.oz = f4.x;
    // object translation (exact zeros when untranslated, as X[3], X[7], X[11] are)
    Q.odx = kTranslated ? q3.x : 0.0f; Q.ody = kTranslated ? q3.y : 0.0f; Q.odz = kTranslated ? q3.z : 0.0f;
    Q.sx = Q.rx > 0; Q.sy = Q.ry > 0; Q.sz = Q.rz > 0;
}

// A leaf item whose triangle record (r0..r2) has arrived: the MT test of
// TD/Trixel.cu:98-145.  kAny: shadow walk (Lmax and the hit triangle come
// from rd[4]).
template <bool kTranslated, bool kCount, bool kAny>
__device__ __forceinline__ void visit_leaf(const Ray& Q, float4 q4, uint4 it, float4 r0, float4 r1, float4 r2,
                                           float4 r3, Visit& o, uint32_t& n_leaf, uint32_t& n_acc) {
    if (kCount) n_leaf++;
    float d = kAny ? q4.z : kDrawDistance;
    uint32_t best = kMiss;
    const bool acc = kTranslated ? leaf_test_rec(Q, r0, r1, r2, it.x & ~kLeafBit, d, best)
                                 : leaf_test_cam(Q, r0, r1, r2, r3, it.x & ~kLeafBit, d, best);
    const bool c = acc && (!kAny || best != __float_as_uint(q4.w));
    o.cand = c;
    o.ctri = best;
    o.key = kAny ? 0ull : ((unsigned long long)__float_as_uint(d) << 32) | code_key(it.w & kCodeMarkMask);
    if (kCount) n_acc += c ? 1u : 0u;
}

// The outcome of an interior node's child ordering (TD/Trixel.cu:146-170):
// the first- and second-popped children's refs and slab values, whether each
// is pushed, and whether the left child is the first.
struct Order {
    uint32_t first, second;
    float f0, f1, g0, g1;
    bool ka, kb, left_first, push_second;
};

// The reference's visit counters of a node's children (kCount renders):
// interior children tested, and descended into.
__device__ __forceinline__ void count_order(const Order& o, uint32_t& n_int, uint32_t& n_desc) {
    const bool first_leaf = (o.first & kLeafBit) != 0, second_leaf = (o.second & kLeafBit) != 0;
    n_int += (first_leaf ? 0u : 1u) + ((o.push_second && !second_leaf) ? 1u : 0u);
    n_desc += ((!first_leaf && o.ka) ? 1u : 0u) + ((o.push_second && !second_leaf && o.kb) ? 1u : 0u);
}

// The child ordering of an interior node whose own slab values are (t0, t1),
// from its child-box record's split word r3 and its children's slab values
// (lt0, lt1) and (rt0, rt1).  kCount: the reference's visit counters of the
// node's children (when `real`).
//
// A value the compiler cannot see through: the double-precision fix-ups of
// tiny s1 values take it, so they stay behind their (rarely taken) uniform
// branches instead of being computed for every record and selected.
__device__ __forceinline__ float opaque(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

// kFast (untranslated walks of rays with normal, nonzero components, under
// the frame proof P.fast): the direction per cut axis is the ray component
// itself (r_a * 1 + r_b * 0 + r_c * 0 == r_a for finite nonzero r), and the
// entry test mint1 >= maxt0 - 1e-16 && maxt0 > -1e-16 (TD/Trixel.cu:146) is
// mint1 >= maxt0: P.fast holds only when every box's maxt0 is >= 2^-20 for
// every ray of the frame (rt_api.cpp fast_proof), where maxt0 - 1e-16 rounds
// to a double above the float below maxt0.
// kAny: a shadow segment's walk, which enters a child box only where the
// segment does: its entry parameter below Lmax (q4.z; root_pass).
template <bool kTranslated, bool kCount, bool kFast = false, bool kAny = false>
__device__ __forceinline__ void order_node(const TraceParams& P, const Ray& Q, float4 q2, float4 q3, float4 q4,
                                           float t0, float t1, float4 r0, float4 r1, float4 r2, float4 r3, float lt0,
                                           float lt1, float rt0, float rt1, bool real, Order& o, uint32_t& n_int,
                                           uint32_t& n_desc) {
    const uint32_t lw = __float_as_uint(r3.z), rw = __float_as_uint(r3.w);
    const uint32_t axis = (lw >> kAxisShift) & 3u;
    const uint32_t L = lw & ~(3u << kAxisShift), Rr = rw & ~kTinyS1Bit;
    const float dir = kFast ? (axis == 0 ? Q.rx : axis == 1 ? Q.ry : Q.rz) : (axis == 0 ? q2.y : axis == 1 ? q2.z : q2.w);
    const float mx = t0 * dir, mn = t1 * dir;
    // The reference's double-promoted epsilon tests (TD/Trixel.cu:146-157):
    // against s2 through the record's exact float thresholds (k_cam_nodes)
    // unless the object is translated
    const float s1r = rec_s1(r0, r1, axis);
    float s1;
    bool left_first, pa;
    if (kTranslated) {
        const float ds = axis == 0 ? q3.w : axis == 1 ? q4.x : q4.y;
        s1 = (float)((double)s1r + kEps + (double)ds);
        const float s2 = rec_s2(r1, r2, axis) + ds;
        left_first = pred::lt_eps_ref(mx, s2);
        pa = pred::gt_eps_ref(mn, s2);
    } else {
        left_first = mx < r3.y;
        pa = mn > r3.x;
        if (kFast) {
            // (float)((double)s1 + 1e-16) == s1 unless s1 is tiny (the
            // record's flag; the camera's P.tiny_s1 says whether any is):
            // the double form for those, behind a wave-uniform branch
            s1 = s1r;
            if (P.tiny_s1) {
                const bool tiny = (rw & kTinyS1Bit) != 0;
                if (__ballot(tiny) != 0ull) s1 = tiny ? pred::add_eps_ref(opaque(s1r)) : s1r;
            }
        } else {
            s1 = pred::add_eps_ref(s1r);
        }
    }
    // every term computed, then selected (no exec-mask branches)
    const bool pb = (mn < s1) | (mx < s1);
    const bool push_second = (left_first & pa) | (!left_first & pb);
    const bool lpass = (kFast ? lt1 >= lt0 : pred::enter_ref(lt0, lt1)) && (!kAny || !RT_SHADOW_SEGMENT || lt0 < q4.z);
    const bool rpass = (kFast ? rt1 >= rt0 : pred::enter_ref(rt0, rt1)) && (!kAny || !RT_SHADOW_SEGMENT || rt0 < q4.z);
    const uint32_t first = left_first ? L : Rr;
    const uint32_t second = left_first ? Rr : L;
    const bool first_leaf = (first & kLeafBit) != 0, second_leaf = (second & kLeafBit) != 0;
    const bool keep_first = first_leaf || (left_first ? lpass : rpass);
    const bool keep_second = push_second && (second_leaf || (left_first ? rpass : lpass));
    o.first = first;
    o.second = second;
    o.f0 = left_first ? lt0 : rt0; o.f1 = left_first ? lt1 : rt1;
    o.g0 = left_first ? rt0 : lt0; o.g1 = left_first ? rt1 : lt1;
    o.ka = keep_first;
    o.kb = keep_second;
    o.left_first = left_first;
    o.push_second = push_second;
    if (kCount && real) count_order(o, n_int, n_desc);
}

// The slab parameters of an interior record's two child boxes (r0..r2).
template <bool kFast>
__device__ __forceinline__ void child_slabs(const Ray& Q, float4 r0, float4 r1, float4 r2, float& lt0, float& lt1,
                                            float& rt0, float& rt1) {
    if (kFast) {
        slab_fast(f2v{r0.x, r0.y}, f2v{r0.z, r0.w}, f2v{r1.x, r1.y}, Q.ix, Q.iy, Q.iz, lt0, lt1);
        slab_fast(f2v{r1.z, r1.w}, f2v{r2.x, r2.y}, f2v{r2.z, r2.w}, Q.ix, Q.iy, Q.iz, rt0, rt1);
    } else {
        slab_vals(Q, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, lt0, lt1);
        slab_vals(Q, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w, rt0, rt1);
    }
}

// An interior item whose child-box record (r0..r3) has arrived: the node's
// child ordering (TD/Trixel.cu:146-170) and the children's slab tests.
template <bool kTranslated, bool kCount, bool kFast = false, bool kAny = false>
__device__ __forceinline__ void visit_interior(const TraceParams& P, const Ray& Q, float4 q2, float4 q3, float4 q4,
                                               uint4 it, float4 r0, float4 r1, float4 r2, float4 r3, Visit& o,
                                               uint32_t& n_int, uint32_t& n_desc) {
    const uint32_t ray = it.w >> 26;
    const uint32_t marked = it.w & kCodeMarkMask;
    // children's slab parameters from the boxes in this record
    float lt0, lt1, rt0, rt1;
    child_slabs<kFast>(Q, r0, r1, r2, lt0, lt1, rt0, rt1);
    Order od;
    order_node<kTranslated, kCount, kFast, kAny>(P, Q, q2, q3, q4, __uint_as_float(it.y), __uint_as_float(it.z), r0, r1, r2,
                                           r3, lt0, lt1, rt0, rt1, true, od, n_int, n_desc);
    const uint32_t meta_first = (ray << 26) | (marked << 1);
    const uint32_t meta_second = meta_first | 1u;
    o.ca = make_uint4(od.first, __float_as_uint(od.f0), __float_as_uint(od.f1), meta_first);
    o.cb = make_uint4(od.second, __float_as_uint(od.g0), __float_as_uint(od.g1), meta_second);
    o.ka = od.ka;
    o.kb = od.kb;
}

// Visits one item whose record has arrived: a leaf's MT test or an interior
// node's child ordering and slab tests.
template <int kStride, bool kTranslated, bool kCount, bool kAny, bool kFast = false, bool kOdP = false>
__device__ __forceinline__ void visit_item(const TraceParams& P, const float2* rd, uint4 it, float4 r0, float4 r1,
                                           float4 r2, float4 r3, Visit& o, uint32_t& n_int, uint32_t& n_leaf,
                                           uint32_t& n_acc, uint32_t& n_desc) {
    Ray Q;
    float4 q2, q3, q4;
    // each path reads its own ray fields (read once before the branch, they
    // spilled 3 VGPRs of the 16-ray instance, no faster)
    if (it.x & kLeafBit) {
        ray_of<kTranslated, kStride, kFast, kOdP>(rd, Q, q2, q3, q4, P.xf);
        visit_leaf<kTranslated, kCount, kAny>(Q, q4, it, r0, r1, r2, r3, o, n_leaf, n_acc);
    } else {
        ray_of<kTranslated, kStride, kFast, kOdP>(rd, Q, q2, q3, q4, P.xf);
        visit_interior<kTranslated, kCount, kFast, kAny>(P, Q, q2, q3, q4, it, r0, r1, r2, r3, o, n_int, n_desc);
    }
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long b) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// One visited item's candidate: any-hit marks the ray; nearest-hit takes the
// 64-bit min of (w, path code) and the unique holder of the minimum records
// its triangle.
template <bool kAny>
__device__ __forceinline__ void record_candidate(unsigned long long* s_key, uint32_t* s_tri, const uint4& it,
                                                 const Visit& v) {
    const uint32_t ray = it.w >> 26;
    if (kAny) {
        if (v.cand) s_key[ray] = 0ull;
    } else {
        if (v.cand) atomicMin(&s_key[ray], v.key);
        __builtin_amdgcn_wave_barrier();
        if (v.cand && s_key[ray] == v.key) s_tri[ray] = v.ctri;
    }
}

// Pushes one visited item's children (ballot compaction) at items[at...];
// returns how many the wave pushed.  The order decides which items the next
// pops take when the pool holds more than one pop.  Nearest-hit walks visit
// every intersected node whatever the order; they push all lanes' first
// children, then all second ones (0.084 ms at 1080p vs 0.092 for per-lane
// pairs).  Any-hit (shadow) walks stop at the first occluder, and which order
// reaches it soonest depends on the scene and resolution, so
// it is a template choice of the launch (the host times the four and keeps
// the fastest): 0 as nearest-hit, 1 per-lane pairs (first, second), 2 all
// second children then all first ones (first children on top), 3 per-lane
// pairs (second, first).  A runtime order costs scratch spills (measured).
template <bool kAny, int any_order>
__device__ __forceinline__ int push_children(uint4* items, int at, const Visit& v) {
    const unsigned long long m1 = __ballot(v.ka), m2 = __ballot(v.kb);
    const int n1 = __builtin_popcountll(m1), n2 = __builtin_popcountll(m2);
    constexpr int ord = kAny ? any_order : 0;
    if (ord & 1) {   // per-lane pairs
        const int off = (int)(lanes_below(m1) + lanes_below(m2));
        if (ord == 1) {
            if (v.ka) items[at + off] = v.ca;
            if (v.kb) items[at + off + (v.ka ? 1 : 0)] = v.cb;
        } else {
            if (v.kb) items[at + off] = v.cb;
            if (v.ka) items[at + off + (v.kb ? 1 : 0)] = v.ca;
        }
    } else if (ord == 2) {
        if (v.kb) items[at + (int)lanes_below(m2)] = v.cb;
        if (v.ka) items[at + n2 + (int)lanes_below(m1)] = v.ca;
    } else {
        if (v.ka) items[at + (int)lanes_below(m1)] = v.ca;
        if (v.kb) items[at + n1 + (int)lanes_below(m2)] = v.cb;
    }
    return n1 + n2;
}

// One slot of a kFast one-level pool iteration (nearest-hit walks): the
// item `it` of each lane (act: the lane holds one) whose record r0..r3 has
// arrived, its visit, its candidate, and the pushes of the children, at
// items[at...]; returns how many the wave pushed.  The child ordering's
// booleans are wave lane masks (ballots of the compares, combined by scalar
// ops), and the pushes store under those masks: all left children, then all
// right ones, each carrying its DFS path bit (0 for the child the reference
// pops first).  Which children are visited, and each item's path code, are
// the reference's (TD/Trixel.cu:146-170); only the pool order differs, and
// the nearest hit does not depend on it.
// The first three fields of the items' rays (kFast walks).  A 32-ray wave's
// lanes read up to 32 distinct rays: one 8-byte field of each is 256 bytes,
// one pass over the 64 banks, so each field is its own ds_read_b64 (merged
// into a ds_read2_b64 the two fields take two passes, counted as bank
// conflicts: 0.47-0.75 conflict cycles per LDS instruction at C3).
#ifndef RT_RAY_READ_SPLIT
#define RT_RAY_READ_SPLIT 1
#endif
template <int kStride>
__device__ __forceinline__ void ray_fields3(const float2* rd, float2& f0, float2& f1, float2& f2) {
    if (RT_RAY_READ_SPLIT && kStride == RT_RAY_STRIDE32) {
        f0 = rd[0];
        asm volatile("" ::: "memory");
        f1 = rd[kStride];
        asm volatile("" ::: "memory");
        f2 = rd[2 * kStride];
    } else {
        f0 = rd[0];
        f1 = rd[kStride];
        f2 = rd[2 * kStride];
    }
}

template <int kStride, bool kCount, int kOct = 8>
__device__ __forceinline__ int fast_slot(const TraceParams& P, uint4* items, int at, const float2* s_ray,
                                         unsigned long long* s_key, uint32_t* s_tri, uint4 it, bool act, float4 r0,
                                         float4 r1, float4 r2, float4 r3, uint32_t& n_int, uint32_t& n_leaf,
                                         uint32_t& n_acc, uint32_t& n_desc) {
    // The leaf and the interior code each run behind a wave-uniform branch
    // (taken when some lane holds that kind) with every lane computing, and
    // their results are masked by the kind: no exec-mask bookkeeping, and the
    // ballots of the ordering stay scalar.  A lane of the other kind reads
    // its own record as this kind's (plain floats; its results are dropped).
    const float2* rd = s_ray + (size_t)(it.w >> 26);
    const unsigned long long A = __ballot(act), LEAF = __ballot((it.x & kLeafBit) != 0) & A, INT = A & ~LEAF;
    float2 f0, f1, f2;
    ray_fields3<kStride>(rd, f0, f1, f2);
    const float rx = f0.x, ry = f0.y, rz = f1.x, ix = f1.y, iy = f2.x, iz = f2.y;
    Visit v;
    v.cand = false;
    if (LEAF) {
        Ray Q;
        Q.rx = rx; Q.ry = ry; Q.rz = rz;
        uint32_t nl = 0, na = 0;
        visit_leaf<false, kCount, false>(Q, make_float4(0.0f, 0.0f, 0.0f, 0.0f), it, r0, r1, r2, r3, v, nl, na);
        const bool mine = __builtin_amdgcn_inverse_ballot_w64(LEAF);
        v.cand = v.cand && mine;
        if (kCount) {
            n_leaf += mine ? nl : 0u;
            n_acc += mine ? na : 0u;
        }
        record_candidate<false>(s_key, s_tri, it, v);
    }
    if (!INT) return 0;
    float lt0, lt1, rt0, rt1;
    slab_pair_oct<kOct>(r0, r1, r2, ix, iy, iz, lt0, lt1, rt0, rt1);
    const uint32_t lw = __float_as_uint(r3.z), rw = __float_as_uint(r3.w);
    const uint32_t axis = (lw >> kAxisShift) & 3u;
    const uint32_t L = lw & ~(3u << kAxisShift), R = rw & ~kTinyS1Bit;
    // the direction on the cut axis is the component itself (order_node)
    const float dir = axis == 2 ? rz : axis == 1 ? ry : rx;
    const float t0 = __uint_as_float(it.y), t1 = __uint_as_float(it.z);
    const float mx = t0 * dir, mn = t1 * dir;
    float s1 = rec_s1(r0, r1, axis);
    if (P.tiny_s1) {  // (a scalar branch; inside, the double form for every lane and a select)
        const float s1t = pred::add_eps_ref(opaque(s1));
        s1 = (rw & kTinyS1Bit) != 0 ? s1t : s1;
    }
    // TD/Trixel.cu:146-168 as lane masks: left first (maxt0 < s2 + eps),
    // the second child pushed (mint1 > s2 - eps, or below s1), each child
    // kept when a leaf or entered (the kFast entry test)
    const bool lf = mx < r3.y;
    const unsigned long long LF = __ballot(lf);
    const unsigned long long PS = (LF & __ballot(mn > r3.x)) | (~LF & __ballot(fminf(mn, mx) < s1));
    // (each ballot of one compare: a ballot of an or-ed lane mask makes the
    // compiler rebuild it from a 0/1 VGPR)
    const unsigned long long mL = INT & (__ballot(lt1 >= lt0) | __ballot((int32_t)L < 0)) & (LF | PS);
    const unsigned long long mR = INT & (__ballot(rt1 >= rt0) | __ballot((int32_t)R < 0)) & (~LF | PS);
    // the children's marked code: the item's shifted up a level (marked <
    // 2^25, so adding it to the word is the shift)
    const uint32_t meta = it.w + (it.w & kCodeMarkMask);
    if (kCount && __builtin_amdgcn_inverse_ballot_w64(INT)) {  // the reference's counters (count_order)
        const bool ps = __builtin_amdgcn_inverse_ballot_w64(PS);
        const bool li = (L & kLeafBit) == 0, ri = (R & kLeafBit) == 0, lp = lt1 >= lt0, rp = rt1 >= rt0;
        const bool fi = lf ? li : ri, si = lf ? ri : li, fp = lf ? lp : rp, sp = lf ? rp : lp;
        n_int += (fi ? 1u : 0u) + ((ps && si) ? 1u : 0u);
        n_desc += ((fi && fp) ? 1u : 0u) + ((ps && si && sp) ? 1u : 0u);
    }
    // all left children, then all right ones, each with its path bit
    const int nL = __builtin_popcountll(mL);
    if (__builtin_amdgcn_inverse_ballot_w64(mL))
        items[at + (int)lanes_below(mL)] = make_uint4(L, __float_as_uint(lt0), __float_as_uint(lt1), meta | (lf ? 0u : 1u));
    if (__builtin_amdgcn_inverse_ballot_w64(mR))
        items[at + nL + (int)lanes_below(mR)] =
            make_uint4(R, __float_as_uint(rt0), __float_as_uint(rt1), meta | (lf ? 1u : 0u));
    return nL + __builtin_popcountll(mR);
}

// One slot of a translated kFast pool iteration (round 6, verdict r05 items
// 2-3): the walks of an object moved by an offset (its rays carry the
// translation od, TD/Trixel.cu:60-66,94-95) and the shadow walks from the
// light (od = (-2, -2, -2), a12), under a proof that every box's entry
// parameter is >= 2^-20 for each of their rays (rt_api.cpp fast_proof for the
// frame; fast_proof_shadow for the light plus trace_unit's per-wave sign
// check).  The reference's tests, exactly, in single precision:
//   * entry (TD/Trixel.cu:146): mint1 >= maxt0 (maxt0 >= 2^-20, as kFast);
//   * the child order against s2 + ds (:155-157): s = s2 + ds is the
//     reference's float sum, and for |s| >= 2^-20 the double compares are
//     pred::lt_eps_x / gt_eps_x (the equality case included); a lane whose s
//     is tiny takes the double form behind a wave-uniform branch;
//   * s1 + 1e-16 + ds (:150-151): the reference's double expression;
//   * slabs with the offsets (slab_pair_xoct), the MT test leaf_test_xf.
// The direction on the cut axis is the component itself and ds the offset's
// component (r_a * 1 + r_b * 0 + r_c * 0 == r_a for finite nonzero r; a zero
// offset component's sign does not reach any compare).  kAny: the shadow
// walk (Lmax and the hit triangle from field 9, no path codes; pushes in
// the launch's any-hit order kAnyOrd, push_children).  Nearest-hit walks
// push as fast_slot does.
template <int kStride, bool kCount, bool kAny, int kAnyOrd, int kOct, bool kOdP = false>
__device__ __forceinline__ int xfast_slot(const TraceParams& P, uint4* items, int at, const float2* s_ray,
                                          unsigned long long* s_key, uint32_t* s_tri, uint4 it, bool act, float4 r0,
                                          float4 r1, float4 r2, float4 r3, uint32_t& n_int, uint32_t& n_leaf,
                                          uint32_t& n_acc, uint32_t& n_desc) {
    const float2* rd = s_ray + (size_t)(it.w >> 26);
    const unsigned long long A = __ballot(act), LEAF = __ballot((it.x & kLeafBit) != 0) & A, INT = A & ~LEAF;
    const float2 f0 = rd[0], f1 = rd[kStride], f2 = rd[2 * kStride];
    const float2 f6 = kOdP ? make_float2(P.xf[3], P.xf[7]) : rd[6 * kStride];
    const float2 f7 = kOdP ? make_float2(P.xf[11], 0.0f) : rd[7 * kStride];
    const float rx = f0.x, ry = f0.y, rz = f1.x, ix = f1.y, iy = f2.x, iz = f2.y;
    const float odx = f6.x, ody = f6.y, odz = f7.x;
    if (LEAF) {
        Ray Q;
        Q.rx = rx; Q.ry = ry; Q.rz = rz;
        Q.odx = odx; Q.ody = ody; Q.odz = odz;
        const float2 f9 = kAny ? rd[9 * kStride] : make_float2(0.0f, 0.0f);
        float d = kAny ? f9.x : kDrawDistance;
        uint32_t best = kMiss;
        const bool acc = leaf_test_xf(Q, r0, r1, r2, it.x & ~kLeafBit, d, best);
        const bool mine = __builtin_amdgcn_inverse_ballot_w64(LEAF);
        Visit v;
        v.cand = acc && mine && (!kAny || best != __float_as_uint(f9.y));
        v.ctri = best;
        v.key = kAny ? 0ull : ((unsigned long long)__float_as_uint(d) << 32) | code_key(it.w & kCodeMarkMask);
        if (kCount) {
            n_leaf += mine ? 1u : 0u;
            n_acc += v.cand ? 1u : 0u;
        }
        record_candidate<kAny>(s_key, s_tri, it, v);
    }
    if (!INT) return 0;
    const float2 f3 = rd[3 * kStride], f4 = rd[4 * kStride];
    float lt0, lt1, rt0, rt1;
    slab_pair_xoct<kOct>(r0, r1, r2, ix, iy, iz, f3.x, f3.y, f4.x, lt0, lt1, rt0, rt1);
    // a shadow segment enters a box only below Lmax (root_pass): the exit
    // parameter of a box it does not enter is set below its entry
    if constexpr (kAny && RT_SHADOW_SEGMENT) {
        const float lim = rd[9 * kStride].x;
        lt1 = lt0 < lim ? lt1 : -INFINITY;
        rt1 = rt0 < lim ? rt1 : -INFINITY;
    }
    const uint32_t lw = __float_as_uint(r3.z), rw = __float_as_uint(r3.w);
    const uint32_t axis = (lw >> kAxisShift) & 3u;
    const uint32_t L = lw & ~(3u << kAxisShift), R = rw & ~kTinyS1Bit;
    const float dir = axis == 2 ? rz : axis == 1 ? ry : rx;
    const float ds = axis == 2 ? odz : axis == 1 ? ody : odx;
    const float t0 = __uint_as_float(it.y), t1 = __uint_as_float(it.z);
    const float mx = t0 * dir, mn = t1 * dir;
    const float s1 = (float)(((double)rec_s1(r0, r1, axis) + kEps) + (double)ds);
    const float s2 = rec_s2(r1, r2, axis) + ds;
    bool lf = pred::lt_eps_x(mx, s2), pa = pred::gt_eps_x(mn, s2);
    const bool tiny = !(fabsf(s2) >= 0x1p-20f);  // (NaN s2 takes it too: the double form decides)
    if (__ballot(tiny) & INT) {
        lf = tiny ? pred::lt_eps_ref(opaque(mx), s2) : lf;
        pa = tiny ? pred::gt_eps_ref(opaque(mn), s2) : pa;
    }
    const unsigned long long LF = __ballot(lf);
    const unsigned long long PS = (LF & __ballot(pa)) | (~LF & __ballot(fminf(mn, mx) < s1));
    const unsigned long long mL = INT & (__ballot(lt1 >= lt0) | __ballot((int32_t)L < 0)) & (LF | PS);
    const unsigned long long mR = INT & (__ballot(rt1 >= rt0) | __ballot((int32_t)R < 0)) & (~LF | PS);
    if (kCount && __builtin_amdgcn_inverse_ballot_w64(INT)) {  // the reference's counters (count_order)
        const bool ps = __builtin_amdgcn_inverse_ballot_w64(PS);
        const bool li = (L & kLeafBit) == 0, ri = (R & kLeafBit) == 0, lp = lt1 >= lt0, rp = rt1 >= rt0;
        const bool fi = lf ? li : ri, si = lf ? ri : li, fp = lf ? lp : rp, sp = lf ? rp : lp;
        n_int += (fi ? 1u : 0u) + ((ps && si) ? 1u : 0u);
        n_desc += ((fi && fp) ? 1u : 0u) + ((ps && si && sp) ? 1u : 0u);
    }
    if constexpr (kAny) {
        // any-hit: no path codes; the launch's push order over (first, second)
        // (selected field by field: a select of the two uint4 items became a
        // select of their addresses in scratch)
        const bool kl = __builtin_amdgcn_inverse_ballot_w64(mL), kr = __builtin_amdgcn_inverse_ballot_w64(mR);
        const uint32_t l0 = __float_as_uint(lt0), l1 = __float_as_uint(lt1);
        const uint32_t q0 = __float_as_uint(rt0), q1 = __float_as_uint(rt1);
        Visit v;
        v.ca = make_uint4(lf ? L : R, lf ? l0 : q0, lf ? l1 : q1, it.w);
        v.cb = make_uint4(lf ? R : L, lf ? q0 : l0, lf ? q1 : l1, it.w);
        v.ka = lf ? kl : kr;
        v.kb = lf ? kr : kl;
        return push_children<true, kAnyOrd>(items, at, v);
    } else {
        const uint32_t meta = it.w + (it.w & kCodeMarkMask);
        const int nL = __builtin_popcountll(mL);
        if (__builtin_amdgcn_inverse_ballot_w64(mL))
            items[at + (int)lanes_below(mL)] =
                make_uint4(L, __float_as_uint(lt0), __float_as_uint(lt1), meta | (lf ? 0u : 1u));
        if (__builtin_amdgcn_inverse_ballot_w64(mR))
            items[at + nL + (int)lanes_below(mR)] =
                make_uint4(R, __float_as_uint(rt0), __float_as_uint(rt1), meta | (lf ? 1u : 0u));
        return nL + __builtin_popcountll(mR);
    }
}

// Record loads by the lanes that use them only (kFast walks of 8- and 16-ray
// units; RT_MASKED_LOADS32 for 32-ray units).  The walk's busiest unit is the
// vector memory path (r05w: TA busy 0.85, TD busy 0.96 of the knot's cycles),
// whose cost follows the lanes a load instruction carries, not the distinct
// addresses: an idle lane that re-reads a live item's record costs as much
// as a real one, and so does a lane whose buffer load the range check drops
// (r05y).  Exec-masked loads: knot 1080p +3.9 %, dragon 1080p +11 %; 32-ray
// units (C3, knot 960x540), whose walks are HBM-bound, lose 3-4 % (r05z).
// 0: every lane loads (idle lanes a live item's record).
#ifndef RT_MASKED_LOADS
#define RT_MASKED_LOADS 1
#endif
#ifndef RT_MASKED_LOADS32
#define RT_MASKED_LOADS32 0
#endif
template <int kStride>
constexpr bool masked_loads() {
    return kStride == RT_RAY_STRIDE32 ? RT_MASKED_LOADS32 != 0 : RT_MASKED_LOADS != 0;
}

// Record-load statistics (verdict r05 item 1: "measure live lanes per pop
// against distinct nodes per pop, and loads per visit by walk form"), in
// diagnostic builds (-DRT_VMEM_STATS=1, debug bit 16384) only.  Per walk form
// (0 a single-slot pop, 1 / 2 slot 0 / slot 1 of a two-slot pop, 3 a
// two-level iteration) and per record group (four dwordx4 wave loads):
//   [0] groups, [1] live items, [2] loading lanes, [3] the vector memory
//   path's cycles per wave load by tools/ubench_l1.hip's model (sum over the
//   16 lane quads of max(1, distinct 128-B lines its loading lanes touch)),
//   [4] distinct records among the live lanes, [5] distinct 128-B lines.
#ifndef RT_VMEM_STATS
#define RT_VMEM_STATS 0
#endif
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    for (int off = 32; off >= 1; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    return v;
}
__device__ __forceinline__ void vmem_stat(const TraceParams& P, int form, const float4* addr, bool load, bool live) {
    if (!RT_VMEM_STATS || !P.vstat) return;
    const int lane = (int)threadIdx.x & 63;
    const uint32_t off = (uint32_t)((const char*)addr - (const char*)P.inode);
    const uint32_t line = off >> 7, rec = off >> 6;
    const uint32_t v = load ? line : 0xFFFFFFFFu;
    const uint32_t q0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, true);
    const uint32_t q1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xF, 0xF, true);
    const uint32_t q2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xAA, 0xF, 0xF, true);
    const uint32_t q3 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xFF, 0xF, 0xF, true);
    const uint32_t d = (q0 != ~0u ? 1u : 0u) + ((q1 != ~0u && q1 != q0) ? 1u : 0u) +
                       ((q2 != ~0u && q2 != q0 && q2 != q1) ? 1u : 0u) +
                       ((q3 != ~0u && q3 != q0 && q3 != q1 && q3 != q2) ? 1u : 0u);
    const uint32_t qcost = wave_sum_u32((lane & 3) == 0 ? (d > 0 ? d : 1u) : 0u);
    const unsigned long long LIVE = __ballot(live), LOAD = __ballot(load);
    bool first_rec = live, first_line = live;
    for (int j = 0; j < 64; j++) {
        const uint32_t rj = (uint32_t)__builtin_amdgcn_readlane((int)rec, j);
        const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)line, j);
        if (((LIVE >> j) & 1ull) && j < lane) {
            if (rj == rec) first_rec = false;
            if (lj == line) first_line = false;
        }
    }
    if (lane == 0) {
        unsigned long long* c = P.vstat + 6 * form;
        atomicAdd(&c[0], 1ull);
        atomicAdd(&c[1], (unsigned long long)__builtin_popcountll(LIVE));
        atomicAdd(&c[2], (unsigned long long)__builtin_popcountll(LOAD));
        atomicAdd(&c[3], (unsigned long long)qcost);
    }
    const unsigned long long FR = __ballot(first_rec), FL = __ballot(first_line);
    if (lane == 0) {
        atomicAdd(&P.vstat[6 * form + 4], (unsigned long long)__builtin_popcountll(FR));
        atomicAdd(&P.vstat[6 * form + 5], (unsigned long long)__builtin_popcountll(FL));
    }
}

// Two-level pool iterations (default on; debug bit 1024 or a
// non-BFS record order turns them off).  A wave's chain of pool iterations is
// at least the tree's depth, and most iterations pop small pools (24 items on
// average, r03 stamps), so most lanes idle.  When the pool holds at most 16
// items every item is popped and handled by a quad of lanes: role 0 visits
// the item's node as a one-level iteration does (its children's slab tests,
// their order), and roles 1 and 2 load, in the same memory round trip, the
// child-box records of the node's left and right child -- for an interior
// node at depth <= P.two_depth its children are interior records at
// positions 2i + 1 and 2i + 2 (BFS record order, the shape rt_api.cpp's
// two_level_depth checks) -- take their own slab values and the node's order
// from role 0 (DPP quad broadcasts), visit the children the node keeps, and
// push the grandchildren.  So two tree levels of a small pool take one
// iteration of about one level's instructions.  The visited (ray, node) items
// are the reference's, as with any pop order, and so are the counters.
#ifndef RT_TWO_MAX
#define RT_TWO_MAX 16
#endif

// Every lane of a quad receives the value of the quad's lane 0 (DPP
// quad_perm [0,0,0,0]); the exchange runs with every lane active.
__device__ __forceinline__ uint32_t quad_bcast0(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x00, 0xF, 0xF, true);
}
__device__ __forceinline__ float quad_bcast0(float x) { return __uint_as_float(quad_bcast0(__float_as_uint(x))); }

// One two-level iteration over the whole pool (n <= 16 items); returns the
// new pool size (<= 4n: an item pushes its two children or its four
// grandchildren).
template <int kStride, bool kTranslated, bool kCount, bool kAny, int kOrder, bool kFast, bool kOdP = false>
__device__ __forceinline__ int two_level_iter(const TraceParams& P, uint4* items, const float2* s_ray,
                                              unsigned long long* s_key, uint32_t* s_tri, int n, int lane,
                                              uint32_t& n_int, uint32_t& n_leaf, uint32_t& n_acc, uint32_t& n_desc) {
    // the lane's quad and role, recomputed here behind an empty asm so that
    // they are not hoisted out of the pool loop (live across the one-level
    // iterations too, they cost the 16-ray instance a spill)
    int l = lane;
    asm volatile("" : "+v"(l));
    const int k = l >> 2, role = l & 3;  // role 0: the item's node; 1 / 2: its left / right child
    bool act = k < n;
    const uint4 it = items[act ? k : 0];
    __builtin_amdgcn_wave_barrier();
    if (kAny && (!kCount || kOrder >= 4))
        if (act && s_key[it.w >> 26] == 0ull) act = false;
    const uint32_t marked = it.w & kCodeMarkMask;
    const bool interior = (it.x & kLeafBit) == 0;
    const int depth = 31 - __builtin_clz(marked);
    const bool el = act && interior && depth <= P.two_depth;  // the same on the quad's lanes
    const bool child = (role == 1 || role == 2) && el;
    // role 0 (and the idle role 3): the item's record; roles 1, 2: the child's
    const float4* pa = child ? P.inode + 4 * (2 * (size_t)it.x + (size_t)role) : record_of(P, it.x);
    const float4 a0 = pa[0], a1 = pa[1], a2 = pa[2], a3 = pa[3];
    Ray Q;
    float4 q2, q3, q4;
    ray_of<kTranslated, kStride, kFast, kOdP>(s_ray + (size_t)(it.w >> 26), Q, q2, q3, q4, P.xf);
    // the slab values of the record's two child boxes (role 0: the node's
    // children; roles 1, 2: the child's children), then each lane's node's
    // own values: role 0 the item's, roles 1, 2 what role 0 computed for them
    float at0, at1, bt0, bt1;
    child_slabs<kFast>(Q, a0, a1, a2, at0, at1, bt0, bt1);
    const float xl0 = quad_bcast0(at0), xl1 = quad_bcast0(at1), xr0 = quad_bcast0(bt0), xr1 = quad_bcast0(bt1);
    const float t0 = role == 0 ? __uint_as_float(it.y) : role == 1 ? xl0 : xr0;
    const float t1 = role == 0 ? __uint_as_float(it.z) : role == 1 ? xl1 : xr1;
    Order o;
    order_node<kTranslated, kCount, kFast, kAny>(P, Q, q2, q3, q4, t0, t1, a0, a1, a2, a3, at0, at1, bt0, bt1, false, o, n_int,
                                           n_desc);
    // role 0's verdict on its node's children, to roles 1 and 2
    const uint32_t fl = quad_bcast0((o.left_first ? 1u : 0u) | (o.ka ? 2u : 0u) | (o.kb ? 4u : 0u));
    const bool lfirst = (fl & 1u) != 0;
    const bool is_first = (role == 1) == lfirst;  // roles 1, 2: whether this child is popped first
    const bool kept = child && ((fl & (is_first ? 2u : 4u)) != 0);
    // the node this lane visited: role 0's item, or a child role 0 keeps
    const bool real = role == 0 ? (act && interior) : kept;
    if (kCount && real) count_order(o, n_int, n_desc);
    // role 0 pushes its node's children unless roles 1 and 2 expand them
    const bool push = role == 0 ? (act && interior && !el) : kept;
    const uint32_t code = role == 0 ? marked : ((marked << 1) | (is_first ? 0u : 1u));
    const uint32_t meta = ((it.w >> 26) << 26) | (code << 1);
    const bool p1 = push && o.ka, p2 = push && o.kb;
    const unsigned long long m1 = __ballot(p1), m2 = __ballot(p2);
    const int n1 = __builtin_popcountll(m1);
    if (p1) items[(int)lanes_below(m1)] = make_uint4(o.first, __float_as_uint(o.f0), __float_as_uint(o.f1), meta);
    if (p2)
        items[n1 + (int)lanes_below(m2)] = make_uint4(o.second, __float_as_uint(o.g0), __float_as_uint(o.g1), meta | 1u);
    {
        // role 0, a leaf item: the MT test (last: its temporaries and the
        // orders' are not live together)
        Visit v;
        v.ka = v.kb = false; v.cand = false;
        if (role == 0 && act && !interior)
            visit_leaf<kTranslated, kCount, kAny>(Q, q4, it, a0, a1, a2, a3, v, n_leaf, n_acc);
        record_candidate<kAny>(s_key, s_tri, it, v);
    }
    return n1 + __builtin_popcountll(m2);
}

// The two-level iteration of a kFast walk, as lane masks (fast_slot's forms):
// lane 4k + r holds item k; role 0 its node, roles 1 and 2 the node's left
// and right child when the item expands two levels, role 3 the item's node
// again.  Role 3's slab values of the node's right box reach role 2 and role
// 0's of its left box reach role 1 in one quad_perm [0, 0, 3, 3] exchange per
// value; with masked loads (masked_loads) role 3 loads no record and roles 1
// and 2 take both boxes' values from role 0, two exchanges per value.  Which
// nodes are visited and pushed, and every path code, are two_level_iter's.
// kXl (round 6): a translated walk's form (xfast_slot's slabs with the
// offsets, its ordering against s2 + ds, the translated MT test).
template <int kStride, bool kCount, int kOct = 8, bool kXl = false, bool kOdP = false>
__device__ __forceinline__ int two_level_fast(const TraceParams& P, uint4* items, const float2* s_ray,
                                              unsigned long long* s_key, uint32_t* s_tri, int n, int lane,
                                              uint32_t& n_int, uint32_t& n_leaf, uint32_t& n_acc, uint32_t& n_desc) {
    int l = lane;
    asm volatile("" : "+v"(l));
    const int k = l >> 2, role = l & 3;
    const bool act = k < n;
    const uint4 it = items[act ? k : 0];
    __builtin_amdgcn_wave_barrier();
    constexpr unsigned long long R0 = 0x1111111111111111ull;  // the role-0 lanes
    const uint32_t marked = it.w & kCodeMarkMask;
    const bool interior = (it.x & kLeafBit) == 0;
    const int depth = 31 - __builtin_clz(marked);
    // (ballots of single compares, combined by scalar ops)
    const unsigned long long ACT0 = __ballot(act) & R0, INTB = __ballot(interior);
    const unsigned long long INT0 = ACT0 & INTB;
    const unsigned long long EL0 = INT0 & __ballot(depth <= P.two_depth);
    const bool child = __builtin_amdgcn_inverse_ballot_w64((EL0 << 1) | (EL0 << 2));
    const float4* pa = child ? (const float4*)((const char*)P.inode + ((2 * it.x + (uint32_t)role) << 6))
                             : record_fast(P, it.x);
    float4 a0, a1, a2, a3;
    vmem_stat(P, 3, pa, masked_loads<kStride>() ? (role == 0 ? act : child) : true, role == 0 ? act : child);
    if (masked_loads<kStride>()) {
        // only the lanes whose record is used load one: role 0 of a live
        // item, roles 1 and 2 of an expanded one
        if (role == 0 ? act : child) {
            a0 = pa[0]; a1 = pa[1]; a2 = pa[2]; a3 = pa[3];
        }
    } else {
        a0 = pa[0]; a1 = pa[1]; a2 = pa[2]; a3 = pa[3];
    }
    const float2* rd = s_ray + (size_t)(it.w >> 26);
    const float2 f0 = rd[0], f1 = rd[kStride], f2 = rd[2 * kStride];
    const float rx = f0.x, ry = f0.y, rz = f1.x, ix = f1.y, iy = f2.x, iz = f2.y;
    const float2 z2 = make_float2(0.0f, 0.0f);
    const float2 f3 = kXl ? rd[3 * kStride] : z2, f4 = kXl ? rd[4 * kStride] : z2;
    const float2 f6 = kXl ? (kOdP ? make_float2(P.xf[3], P.xf[7]) : rd[6 * kStride]) : z2;
    const float2 f7 = kXl ? (kOdP ? make_float2(P.xf[11], 0.0f) : rd[7 * kStride]) : z2;
    // the record's child boxes; each lane's own node's (t0, t1)
    float lt0, lt1, rt0, rt1;
    if constexpr (kXl)
        slab_pair_xoct<kOct>(a0, a1, a2, ix, iy, iz, f3.x, f3.y, f4.x, lt0, lt1, rt0, rt1);
    else
        slab_pair_oct<kOct>(a0, a1, a2, ix, iy, iz, lt0, lt1, rt0, rt1);
    float x0, x1;
    if (masked_loads<kStride>()) {
        // role 0's values of both boxes, to roles 1 (left) and 2 (right)
        const float bl0 = quad_bcast0(lt0), bl1 = quad_bcast0(lt1), br0 = quad_bcast0(rt0), br1 = quad_bcast0(rt1);
        x0 = role == 1 ? bl0 : br0;
        x1 = role == 1 ? bl1 : br1;
    } else {
        const float u0 = role == 3 ? rt0 : lt0, u1 = role == 3 ? rt1 : lt1;
        x0 = __uint_as_float((uint32_t)__builtin_amdgcn_mov_dpp((int)__float_as_uint(u0), 0xF0, 0xF, 0xF, true));
        x1 = __uint_as_float((uint32_t)__builtin_amdgcn_mov_dpp((int)__float_as_uint(u1), 0xF0, 0xF, 0xF, true));
    }
    const float t0 = role == 0 ? __uint_as_float(it.y) : x0, t1 = role == 0 ? __uint_as_float(it.z) : x1;
    // the order of each lane's node (fast_slot)
    const uint32_t lw = __float_as_uint(a3.z), rw = __float_as_uint(a3.w);
    const uint32_t axis = (lw >> kAxisShift) & 3u;
    const uint32_t L = lw & ~(3u << kAxisShift), R = rw & ~kTinyS1Bit;
    const float dir = axis == 2 ? rz : axis == 1 ? ry : rx;
    const float mx = t0 * dir, mn = t1 * dir;
    float s1;
    bool lf, pgt;
    if constexpr (kXl) {
        // xfast_slot's ordering: s2 + ds (the offset's component) through
        // the exact float compares, s1 + 1e-16 + ds in double
        const float ds = axis == 2 ? f7.x : axis == 1 ? f6.y : f6.x;
        s1 = (float)(((double)rec_s1(a0, a1, axis) + kEps) + (double)ds);
        const float s2 = rec_s2(a1, a2, axis) + ds;
        lf = pred::lt_eps_x(mx, s2);
        pgt = pred::gt_eps_x(mn, s2);
        const bool tiny = !(fabsf(s2) >= 0x1p-20f);
        if (__ballot(tiny)) {
            lf = tiny ? pred::lt_eps_ref(opaque(mx), s2) : lf;
            pgt = tiny ? pred::gt_eps_ref(opaque(mn), s2) : pgt;
        }
    } else {
        s1 = rec_s1(a0, a1, axis);
        if (P.tiny_s1) {
            const float s1t = pred::add_eps_ref(opaque(s1));
            s1 = (rw & kTinyS1Bit) != 0 ? s1t : s1;
        }
        lf = mx < a3.y;
        pgt = mn > a3.x;
    }
    const unsigned long long LF = __ballot(lf);
    const unsigned long long PS = (LF & __ballot(pgt)) | (~LF & __ballot(fminf(mn, mx) < s1));
    const unsigned long long KL = (__ballot(lt1 >= lt0) | __ballot((int32_t)L < 0)) & (LF | PS);
    const unsigned long long KR = (__ballot(rt1 >= rt0) | __ballot((int32_t)R < 0)) & (~LF | PS);
    // the children role 0 keeps are visited by roles 1 and 2
    const unsigned long long KEPT = ((EL0 & KL) << 1) | ((EL0 & KR) << 2);
    const unsigned long long VIS = INT0 | KEPT;
    if (kCount && __builtin_amdgcn_inverse_ballot_w64(VIS)) {  // the reference's counters (count_order)
        const bool ps = __builtin_amdgcn_inverse_ballot_w64(PS);
        const bool li = (L & kLeafBit) == 0, ri = (R & kLeafBit) == 0, lp = lt1 >= lt0, rp = rt1 >= rt0;
        const bool fi = lf ? li : ri, si = lf ? ri : li, fp = lf ? lp : rp, sp = lf ? rp : lp;
        n_int += (fi ? 1u : 0u) + ((ps && si) ? 1u : 0u);
        n_desc += ((fi && fp) ? 1u : 0u) + ((ps && si && sp) ? 1u : 0u);
    }
    // role 0 pushes its node's children unless roles 1 and 2 expand them;
    // a kept child pushes its own.  A child's path bit: 0 for the child the
    // parent pops first (role 1 when the parent's left comes first)
    const unsigned long long PUSH = (INT0 & ~EL0) | KEPT;
    const unsigned long long mL = PUSH & KL, mR = PUSH & KR;
    const unsigned long long LF0 = LF & R0;
    const uint32_t second = __builtin_amdgcn_inverse_ballot_w64(((~LF0 & R0) << 1) | (LF0 << 2)) ? 1u : 0u;
    const uint32_t code = role == 0 ? marked : ((marked << 1) | second);
    const uint32_t meta = (it.w & ~kCodeMarkMask) | (code << 1);
    const int nL = __builtin_popcountll(mL);
    if (__builtin_amdgcn_inverse_ballot_w64(mL))
        items[(int)lanes_below(mL)] = make_uint4(L, __float_as_uint(lt0), __float_as_uint(lt1), meta | (lf ? 0u : 1u));
    if (__builtin_amdgcn_inverse_ballot_w64(mR))
        items[nL + (int)lanes_below(mR)] = make_uint4(R, __float_as_uint(rt0), __float_as_uint(rt1), meta | (lf ? 1u : 0u));
    // role 0, a leaf item: the MT test (last)
    const unsigned long long LEAF0 = ACT0 & ~INTB;
    Visit v;
    v.cand = false;
    if (LEAF0) {
        Ray Q;
        Q.rx = rx; Q.ry = ry; Q.rz = rz;
        uint32_t nlf = 0, na = 0;
        if constexpr (kXl) {
            Q.odx = f6.x; Q.ody = f6.y; Q.odz = f7.x;
            float d = kDrawDistance;
            uint32_t best = kMiss;
            const bool acc = leaf_test_xf(Q, a0, a1, a2, it.x & ~kLeafBit, d, best);
            v.cand = acc;
            v.ctri = best;
            v.key = ((unsigned long long)__float_as_uint(d) << 32) | code_key(it.w & kCodeMarkMask);
            nlf = 1u;
            na = acc ? 1u : 0u;
        } else {
            visit_leaf<false, kCount, false>(Q, make_float4(0.0f, 0.0f, 0.0f, 0.0f), it, a0, a1, a2, a3, v, nlf, na);
        }
        const bool mine = __builtin_amdgcn_inverse_ballot_w64(LEAF0);
        v.cand = v.cand && mine;
        if (kCount) {
            n_leaf += mine ? nlf : 0u;
            n_acc += mine ? na : 0u;
        }
        record_candidate<false>(s_key, s_tri, it, v);
    }
    return nL + __builtin_popcountll(mR);
}

// The pool walk of one wave.  kAny = false: nearest hit per ray, key[ray] =
// min (w, path code), tri[ray] = its triangle.  kAny = true (shadow rays): any
// accepted leaf with w < Lmax other than the ray's own hit triangle sets
// key[ray] = 0; without counters the items of such rays are dropped.
// Each lane pops up to P.items (1 or 2) items per iteration and fetches their
// records together, so a lane keeps two memory round trips in flight.
// Shared record loads (round 6, verdict r05 item 1; RT_SHARED_LOADS).  The
// vector memory path's cost per wave load is the sum over its 16 lane quads
// of max(1, distinct 128-B lines its loading lanes touch) cycles
// (tools/ubench_l1.hip), and a pop's items are runs of the same node for
// coherent rays: at the knot 1080p a single-slot pop's 42 live lanes touch
// 8.9 records on average (tools/vmem_stats.py, profiles/r06/vmem/), yet a run
// that straddles a quad boundary costs that quad a line per run.  So only
// the first lane of each run (consecutive lanes holding the same ref) loads
// the record, and the run's other lanes take its 16 dwords from that lane by
// ds_bpermute (the LDS crossbar, not the vector memory path).  Every lane
// ends up with the record of its own item, as before.
// Measured and off (r06e, one box, against RT_SHARED_LOADS 0): the address
// unit's busy share fell (knot 1080p TA_TA_BUSY 0.77 -> 0.57 per CU cycle)
// but the data unit stayed busy on 0.92-0.95 of the cycles, stalled on the
// L1 more (TD_TC_STALL 0.42 -> 0.49), and the 16 ds_bpermute per slot and
// their waits lengthened every pool iteration: the driver's command 12.44k
// -> 9.98k FPS (exec-masked run-start loads 10.09k), C4 20.7k -> 17.5k, C3
// 78.0k -> 66.1k, C5 2,904 -> 2,393.
#ifndef RT_SHARED_LOADS
#define RT_SHARED_LOADS 0
#endif
// Whether this lane starts a run of equal refs among the active lanes, and
// the lane of the start of its run (byte address for ds_bpermute).
__device__ __forceinline__ bool run_start(uint32_t ref, bool act, int lane, int& leader_addr) {
    const uint32_t key = act ? ref : 0xFFFFFFFFu;  // (no ref is all ones: a leaf's index < 2^31 - 1)
    // the previous lane's key (DPP wave_shr:1; lane 0 gets the all-ones key)
    const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)key, 0x138, 0xF, 0xF, false);
    const bool start = act && (lane == 0 || prev != key);
    const unsigned long long S = __ballot(start);
    const unsigned long long m = S & (~0ull >> (63 - lane));  // starts at or below this lane
    const int lead = m ? 63 - __builtin_clzll(m) : lane;
    leader_addr = lead << 2;
    return start;
}
// RT_SHARED_BUF: the run starts' loads as buffer loads whose other lanes
// read beyond the records (the range check drops them) instead of
// exec-masked global loads -- no exec-mask branch, so the compiler's wait
// counts stay exact and slot 1's loads stay in flight while slot 0 is
// visited (with branches it waits for both groups before slot 0's permutes)
#ifndef RT_SHARED_BUF
#define RT_SHARED_BUF 1
#endif
typedef unsigned int rt_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 as_f4(rt_u32x4 r) {
    return make_float4(__uint_as_float(r.x), __uint_as_float(r.y), __uint_as_float(r.z), __uint_as_float(r.w));
}
// The record of `ref` (record_fast's offset) through the buffer resource of
// the camera's records, or zeros without a memory access when !load.
__device__ __forceinline__ void load_record_buf(__amdgpu_buffer_rsrc_t rsrc, const TraceParams& P, uint32_t ref,
                                                bool load, float4& r0, float4& r1, float4& r2, float4& r3) {
    const uint32_t off = load ? (ref << 6) + ((int32_t)ref < 0 ? P.leaf_off : 0u) : 0x80000000u;
    r0 = as_f4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)off, 0, 0));
    r1 = as_f4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(off + 16u), 0, 0));
    r2 = as_f4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(off + 32u), 0, 0));
    r3 = as_f4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(off + 48u), 0, 0));
}
__device__ __forceinline__ float4 share4(float4 v, int addr) {
    return make_float4(__int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v.x))),
                       __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v.y))),
                       __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v.z))),
                       __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v.w))));
}

// kX (round 6): the translated kFast slots (xfast_slot) for a translated
// nearest-hit walk or a shadow walk whose proof holds; its two-level
// iterations keep the double forms (two_level_iter).
#ifndef RT_XMASKED_LOADS
#define RT_XMASKED_LOADS 1
#endif
// Quad-transposed record loads (round 6, kFast one-level pops): in load j
// the four lanes of a quad fetch the four 16-B quarters of quad lane j's
// 64-B record (lane r the quarter r ^ j), so every quad touches one line per
// load -- the L1 / texture units' floor of 16 quad-cycles per wave load
// (profiles/r06/ubench: a load costs the sum over its quads of the distinct
// lines each touches) -- and a 4 x 4 exchange inside the quad (lane-bit
// selects and DPP xor reads) returns each lane its own record.
#ifndef RT_QUAD_LOADS
#define RT_QUAD_LOADS 0
#endif
template <int kCtrl>
__device__ __forceinline__ float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), kCtrl, 0xF, 0xF, true));
}
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_u(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, kCtrl, 0xF, 0xF, true);
}
// The byte offset of an item's record from P.inode (record_fast).
__device__ __forceinline__ uint32_t rec_off(const TraceParams& P, uint32_t ref) {
    return (ref << 6) + ((int32_t)ref < 0 ? P.leaf_off : 0u);
}
// Load j: quad lane r fetches quarter r ^ j of quad lane j's record (every
// lane of the wave active).
__device__ __forceinline__ void quad_load(const TraceParams& P, uint32_t off, int lane, float4& x0, float4& x1,
                                          float4& x2, float4& x3) {
    const char* base = (const char*)P.inode;
    const uint32_t q = ((uint32_t)lane & 3u) << 4;
    const uint32_t o0 = dpp_u<0x00>(off), o1 = dpp_u<0x55>(off), o2 = dpp_u<0xAA>(off), o3 = dpp_u<0xFF>(off);
    x0 = *(const float4*)(base + o0 + q);
    x1 = *(const float4*)(base + o1 + (q ^ 0x10u));
    x2 = *(const float4*)(base + o2 + (q ^ 0x20u));
    x3 = *(const float4*)(base + o3 + (q ^ 0x30u));
}
// One component of the exchange: lane r holds x_j = (quarter r ^ j of lane
// j's record); y_m = quarter m of lane r's own record = lane (r ^ m)'s
// x_r, read by a DPP xor-m of t_m, where t_m(s) = x_(s ^ m) (selects by the
// lane's bits).
__device__ __forceinline__ void quad_xpose1(float x0, float x1, float x2, float x3, bool b0, bool b1, float& y0,
                                            float& y1, float& y2, float& y3) {
    const float p0 = b0 ? x1 : x0, p1 = b0 ? x0 : x1, p2 = b0 ? x3 : x2, p3 = b0 ? x2 : x3;
    y0 = b1 ? p2 : p0;
    y1 = dpp_f<0xB1>(b1 ? p3 : p1);  // quad_perm [1,0,3,2]
    y2 = dpp_f<0x4E>(b1 ? p0 : p2);  // [2,3,0,1]
    y3 = dpp_f<0x1B>(b1 ? p1 : p3);  // [3,2,1,0]
}
__device__ __forceinline__ void quad_xpose(float4& a0, float4& a1, float4& a2, float4& a3, int lane) {
    const bool b0 = (lane & 1) != 0, b1 = (lane & 2) != 0;
    float4 y0, y1, y2, y3;
    quad_xpose1(a0.x, a1.x, a2.x, a3.x, b0, b1, y0.x, y1.x, y2.x, y3.x);
    quad_xpose1(a0.y, a1.y, a2.y, a3.y, b0, b1, y0.y, y1.y, y2.y, y3.y);
    quad_xpose1(a0.z, a1.z, a2.z, a3.z, b0, b1, y0.z, y1.z, y2.z, y3.z);
    quad_xpose1(a0.w, a1.w, a2.w, a3.w, b0, b1, y0.w, y1.w, y2.w, y3.w);
    a0 = y0; a1 = y1; a2 = y2; a3 = y3;
}
#ifndef RT_SHMASKED_LOADS
#define RT_SHMASKED_LOADS 0
#endif
// the translated walks' two-level iterations in the xfast forms (two_level_fast<kXl>)
#ifndef RT_XTWO_LEVEL
#define RT_XTWO_LEVEL 1
#endif
template <int kCap, int kStride, bool kTranslated, bool kCount, bool kAny, int kOrder = 0, bool kFast = false,
          int kOct = 8, bool kX = false, bool kOdP = false>
__device__ __forceinline__ void pool_walk(const TraceParams& P, uint4* items, const float2* s_ray,
                                          unsigned long long* s_key, uint32_t* s_tri, int n, int lane,
                                          uint32_t& iters, uint32_t& popped, uint32_t& n_int, uint32_t& n_leaf,
                                          uint32_t& n_acc, uint32_t& n_desc) {
    const int cap = min(P.pool_cap, kCap);
    const int slack = P.tree_height + 1;
    // P.items: 1 = one item per lane, 2 = two; 65..128 = two only when the
    // pool holds at least that many (a second slot of few items costs a
    // whole slot's instructions)
    const int two_min = P.items == 1 ? 1 << 30 : P.items == 2 ? 65 : P.items;
    while (n > 0) {
        // a pool of at most RT_TWO_MAX items (and room for 4 children each
        // plus the DFS slack): one two-level iteration over all of it.
        // Nearest-hit walks only: an any-hit (shadow) walk stops a ray at its
        // first occluder, and expanding two levels of every pooled item
        // reaches it later (knot 1080p + shadows 4.59k -> 3.38k FPS, r03r)
        if (!kAny && n <= RT_TWO_MAX && P.two_depth >= 0 && 4 * n <= cap - slack) {
            iters++;
            popped += (uint32_t)n;
            if (kFast && !kAny)
                n = two_level_fast<kStride, kCount, kOct>(P, items, s_ray, s_key, s_tri, n, lane, n_int, n_leaf, n_acc, n_desc);
            else if (kX && !kAny && RT_XTWO_LEVEL)
                n = two_level_fast<kStride, kCount, kOct, true, kOdP>(P, items, s_ray, s_key, s_tri, n, lane, n_int,
                                                                     n_leaf, n_acc, n_desc);
            else
                n = two_level_iter<kStride, kTranslated, kCount, kAny, kOrder, kFast, kOdP>(P, items, s_ray, s_key, s_tri, n,
                                                                              lane, n_int, n_leaf, n_acc, n_desc);
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        // Pop as many items as the pool has room for the children of plus
        // the DFS slack below; a single (DFS-like) pop when there is none.
        // Popping k items pushes at most 2k, so a parallel pop leaves
        // n <= cap - slack; a run of single pops starting at n0 is a DFS of
        // the top item's subtree and never holds more than n0 + height items
        // (slack = height + 1, height <= 24), so the pool never overflows.
        int take = min(min(n, n >= two_min ? 128 : 64), cap - slack - n);
        if (take < 1) take = 1;
        iters++;
        popped += (uint32_t)take;
        const int base = n - take;
        // Both items and both records are read unconditionally (idle lanes
        // re-read item `base`, a live item, whose record is a valid address):
        // with guarded loads hipcc zero-fills the registers of the idle path
        // and waits for the first record before issuing the second.
        bool act0 = lane < take, act1 = lane + 64 < take;
        const uint4 it0 = items[base + (act0 ? lane : 0)];
        const uint4 it1 = items[base + (act1 ? lane + 64 : 0)];
        __builtin_amdgcn_wave_barrier();
        // any-hit: a ray already shadowed needs no more visits (kept when
        // counting, so the counters match the oracle's full walk, unless
        // kOrder >= 4: counters of the walk a timed frame does)
        if (kAny && (!kCount || kOrder >= 4)) {
            if (act0 && s_key[it0.w >> 26] == 0ull) act0 = false;
            if (act1 && s_key[it1.w >> 26] == 0ull) act1 = false;
        }
        // both records in flight before either is consumed
        constexpr bool kFastRec = (kFast && !kAny) || kX;
        constexpr bool kMasked = (kFast && !kAny && masked_loads<kStride>()) ||
                                 (kX && (kAny ? RT_SHMASKED_LOADS != 0 : (RT_XMASKED_LOADS != 0 && masked_loads<kStride>())));
        const float4* p0 = kFastRec ? record_fast(P, it0.x) : record_of(P, it0.x);
        const float4* p1 = kFastRec ? record_fast(P, it1.x) : record_of(P, it1.x);
        float4 a0, a1, a2, a3, b0, b1, b2, b3;
        constexpr bool kShared = RT_SHARED_LOADS != 0 && kFastRec;
        constexpr bool kQuad = RT_QUAD_LOADS != 0 && kFast && !kAny && !kX && !kShared;
        int lead0 = 0, lead1 = 0;
        bool st0 = false, st1 = false;
        if (kShared) {
            st0 = run_start(it0.x, act0, lane, lead0);
            if (take > 64) st1 = run_start(it1.x, act1, lane, lead1);
        }
        if (take > 64) {
            vmem_stat(P, 1, p0, kShared ? st0 : true, act0);
            vmem_stat(P, 2, p1, kShared ? st1 : true, act1);
        } else {
            vmem_stat(P, 0, p0, kShared ? st0 : kMasked ? act0 : true, act0);
        }
        if (kQuad) {
            // every lane (idle ones re-read item base's record, a valid one)
            quad_load(P, rec_off(P, it0.x), lane, a0, a1, a2, a3);
            if (take > 64) quad_load(P, rec_off(P, it1.x), lane, b0, b1, b2, b3);
        } else if (kShared && RT_SHARED_BUF) {
            // the run starts load; the other lanes take their run start's
            // record (below, by ds_bpermute).  The resource spans the
            // camera's records (inode, then trec at leaf_off; < 4 GiB)
            const __amdgpu_buffer_rsrc_t rsrc =
                __builtin_amdgcn_make_buffer_rsrc((void*)P.inode, (short)0, (int)P.rec_bytes, 0x00020000);
            load_record_buf(rsrc, P, it0.x, st0, a0, a1, a2, a3);
            if (take > 64) load_record_buf(rsrc, P, it1.x, st1, b0, b1, b2, b3);
        } else if (kShared) {
            if (st0) {
                a0 = p0[0]; a1 = p0[1]; a2 = p0[2]; a3 = p0[3];
            }
            if (take > 64 && st1) {
                b0 = p1[0]; b1 = p1[1]; b2 = p1[2]; b3 = p1[3];
            }
        } else if (kMasked) {
            // a pop of more than 64 items fills slot 0: both slots load on
            // every lane, issued together; a smaller pop loads slot 0's live
            // lanes only (an exec-masked second group waits for the first
            // group's loads before it issues: 32-ray C3 -9 %, r05x)
            if (take > 64) {
                a0 = p0[0]; a1 = p0[1]; a2 = p0[2]; a3 = p0[3];
                b0 = p1[0]; b1 = p1[1]; b2 = p1[2]; b3 = p1[3];
            } else if (act0) {
                a0 = p0[0]; a1 = p0[1]; a2 = p0[2]; a3 = p0[3];
            }
        } else {
            a0 = p0[0]; a1 = p0[1]; a2 = p0[2]; a3 = p0[3];
            b0 = p1[0]; b1 = p1[1]; b2 = p1[2]; b3 = p1[3];
        }
        RT_RECORD_FENCE();
        if (kQuad) quad_xpose(a0, a1, a2, a3, lane);
        if (kShared) {
            a0 = share4(a0, lead0); a1 = share4(a1, lead0); a2 = share4(a2, lead0); a3 = share4(a3, lead0);
        }
        // item 0 is visited, recorded and pushed before item 1 is visited, so
        // its results die before item 1's are made (fewer live VGPRs)
        int total = 0;
        if (kFast && !kAny) {
            total = fast_slot<kStride, kCount, kOct>(P, items, base, s_ray, s_key, s_tri, it0, act0, a0, a1, a2, a3, n_int,
                                               n_leaf, n_acc, n_desc);
            if (take > 64) {
                if (kQuad) quad_xpose(b0, b1, b2, b3, lane);
                if (kShared) {
                    b0 = share4(b0, lead1); b1 = share4(b1, lead1); b2 = share4(b2, lead1); b3 = share4(b3, lead1);
                }
                total += fast_slot<kStride, kCount, kOct>(P, items, base + total, s_ray, s_key, s_tri, it1, act1, b0, b1, b2,
                                                    b3, n_int, n_leaf, n_acc, n_desc);
            }
        } else if (kX) {
            total = xfast_slot<kStride, kCount, kAny, (kOrder & 3), kOct, kOdP>(P, items, base, s_ray, s_key, s_tri, it0, act0, a0,
                                                                       a1, a2, a3, n_int, n_leaf, n_acc, n_desc);
            if (take > 64) {
                if (kShared) {
                    b0 = share4(b0, lead1); b1 = share4(b1, lead1); b2 = share4(b2, lead1); b3 = share4(b3, lead1);
                }
                total += xfast_slot<kStride, kCount, kAny, (kOrder & 3), kOct, kOdP>(P, items, base + total, s_ray, s_key, s_tri,
                                                                            it1, act1, b0, b1, b2, b3, n_int, n_leaf,
                                                                            n_acc, n_desc);
            }
        } else {
        {
            Visit v0;
            v0.ka = v0.kb = false; v0.cand = false;
            if (act0)
                visit_item<kStride, kTranslated, kCount, kAny, kFast, kOdP>(P, s_ray + (size_t)(it0.w >> 26), it0, a0, a1, a2,
                                                                      a3, v0, n_int, n_leaf, n_acc, n_desc);
            record_candidate<kAny>(s_key, s_tri, it0, v0);
            total += push_children<kAny, (kOrder & 3)>(items, base + total, v0);
        }
        // take is wave-uniform: a pop of at most 64 items leaves slot 1 empty
        // on every lane, and skipping its bookkeeping (candidate, ballots,
        // push) outright saves ~300 cycles of such an iteration
        if (take > 64) {
            Visit v1;
            v1.ka = v1.kb = false; v1.cand = false;
            if (act1)
                visit_item<kStride, kTranslated, kCount, kAny, kFast, kOdP>(P, s_ray + (size_t)(it1.w >> 26), it1, b0, b1, b2,
                                                                      b3, v1, n_int, n_leaf, n_acc, n_desc);
            record_candidate<kAny>(s_key, s_tri, it1, v1);
            total += push_children<kAny, (kOrder & 3)>(items, base + total, v1);
        }
        }
        if (base + total > cap) {  // unreachable by the pop rule above; guard anyway
            if (lane == 0) atomicOr(P.err, 2);
            break;
        }
        n = base + total;
        __builtin_amdgcn_wave_barrier();
    }
}

// One instance of the shadow walk per octant of its rays (round 6; the
// primary walk's RT_OCT_WALKS): the slab_pair_xoct near / far selects are
// compile-time.  C5 3,783 -> 3,838 FPS, knot + shadows 6,276 -> 6,369,
// dragon + shadows 9,092 -> 9,203 (r06r, interleaved).
#ifndef RT_SH_OCT
#define RT_SH_OCT 1
#endif
// The root's visit folded into the seeding of kFast walks (trace_unit).
#ifndef RT_ROOT_VISIT
#define RT_ROOT_VISIT 1
#endif
// ... and of translated primary walks: off, measured 1.4-1.7 % slower on the
// moving scenes (r06h; primary +1.5-1.9 %, shadow +0.8-1.0 %), cause not
// isolated
#ifndef RT_XROOT_VISIT
#define RT_XROOT_VISIT 0
#endif
// The root record, the same for every lane, through the constant address
// space (a uniform address there compiles to scalar loads).
__device__ __forceinline__ void root_record(const TraceParams& P, float4& q0, float4& q1, float4& q2, float4& q3) {
    typedef const __attribute__((address_space(4))) float cfloat;
    cfloat* rr = (cfloat*)(P.inode + 4 * (size_t)P.root_ref);
    q0 = make_float4(rr[0], rr[1], rr[2], rr[3]);
    q1 = make_float4(rr[4], rr[5], rr[6], rr[7]);
    q2 = make_float4(rr[8], rr[9], rr[10], rr[11]);
    q3 = make_float4(rr[12], rr[13], rr[14], rr[15]);
}

// Per-wave LDS of the wave-cooperative kernel.
template <int kRays, int kCap, int kRayVec>
struct WaveLds {
    uint4 items[kCap];
    float2 ray[RayLayout<kRays>::kStride * kRayVec * 2];
    unsigned long long key[kRays];
    uint32_t tri[kRays];
    float rn[kRays];  // each ray's rsqrt21 factor, for the shading's second camera_ray
};

struct Counts {
    uint32_t n_int = 0, n_leaf = 0, n_acc = 0, n_desc = 0, n_hit = 0;
};

// A traced pixel's output: Phong of its nearest hit (color_cam_cuda,
// TD/Camera.cu:27-60), black when its shadow ray is occluded, else the
// background; and the hit index.
template <bool kWriteHit, bool kCount>
__device__ __forceinline__ void shade_out(const TraceParams& P, const Pixel& px, const Ray& R, const float cam[3],
                                          unsigned long long kbest, uint32_t best, bool shadowed, Counts& C) {
    const float* X = P.xf;
    uint32_t argb = kBackground;
    if (shadowed) {
        argb = 0x00000000u;  // point_rad stays 0: 0/0 -> (u8)NaN = 0 (H14)
    } else if (best != kMiss) {
        const float d = __uint_as_float((uint32_t)(kbest >> 32));
        const float4 N = P.shade[2 * (size_t)best];
        const float4 M = P.shade[2 * (size_t)best + 1];
        const float pnt[3] = {d * R.rx + R.odx, d * R.ry + R.ody, d * R.rz + R.odz};
        // norm.device_rotate(rot_m, i, -1), TD/vector.cuh:23-33
        const float ax = -1 * N.x, ay = -1 * N.y, az = -1 * N.z;
        const float nrm[3] = {(ax * X[0] + ay * X[1] + az * X[2]) * -1,
                              (ax * X[4] + ay * X[5] + az * X[6]) * -1,
                              (ax * X[8] + ay * X[9] + az * X[10]) * -1};
        const float rad[3] = {M.x, M.y, M.z};
        argb = phong(pnt, nrm, cam, rad);
    }
    put_pixel(P, px.out, argb, best != kMiss);
    if (kWriteHit) P.hit[px.out] = best == kMiss ? (int64_t)-1 : (int64_t)best;
    if (kCount && best != kMiss) C.n_hit++;
}

// One wave's unit of work: the kRays pixels (8 x kRays/8) of unit U.
constexpr size_t kNoDbg = ~(size_t)0;
constexpr int kCoarseMax = 32;  // coarse groups per wave (RT_OPT_COARSE <= 32)
template <int kRays, int kCap, int kRayVec, bool kTranslated, bool kWriteHit, bool kCount, int kShadow>
__device__ __forceinline__ void trace_unit(const TraceParams& P, WaveLds<kRays, kCap, kRayVec>& S_, const Unit& U,
                                           int lane, size_t dbg_slot, uint32_t* cost, Counts& C,
                                           int32_t nrows = kRays / 8, int32_t ncols = 8) {
    using RL = RayLayout<kRays>;
    // a translated instance without shadow rays keeps six ray fields in LDS
    // and reads the offset from the transform (ray_of kOdP; round 6)
    constexpr bool kOdP = kTranslated && kRayVec == 3;
    uint4* items = S_.items;
    Pixel px;
    bool live = unit_pixel(P, U, nrows, lane, px, ncols);  // every lane stays for the ballots
    const unsigned long long t_start = P.dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
    uint32_t iters = 0, popped = 0;

    int n;
    bool fast;  // the walk takes the kFast forms (slab_fast, order_node)
    int oct = 8;  // the octant every live ray of the unit lies in (slab_pair_oct), 8 = mixed
    {
        // the ray goes to LDS for the walk; shading recomputes it afterwards
        // (the same float expressions), so it is not live across the walk
        float cam0[3];
        Ray R0;
        float rn0 = 1.0f;
        camera_ray<false, !kTranslated>(P, px, live, cam0, R0, rn0);
        // every live ray's components normal and nonzero (1/r finite), under
        // the frame proof P.fast (rt_api.cpp)
        // (translated walks: the xfast_slot forms under the same proof,
        // whose margins cover the offsets, rt_api.cpp fast_proof)
        fast = P.fast && __ballot(live && !(fabsf(R0.rx) >= 0x1p-126f && fabsf(R0.ry) >= 0x1p-126f &&
                                            fabsf(R0.rz) >= 0x1p-126f)) == 0ull;
        if (RT_OCT_WALKS && fast) {  // (the octant of the object-space rays)
            const unsigned long long LV = __ballot(live), PX = __ballot(live && R0.rx > 0.0f),
                                     PY = __ballot(live && R0.ry > 0.0f), PZ = __ballot(live && R0.rz > 0.0f);
            if ((PX == 0ull || PX == LV) && (PY == 0ull || PY == LV) && (PZ == 0ull || PZ == LV))
                oct = (PX == LV ? 1 : 0) | (PY == LV ? 2 : 0) | (PZ == LV ? 4 : 0);
        }
        if (lane < kRays) {
            store_ray(&S_.ray[lane], RL::kStride, R0, kTranslated && !kOdP, 0.0f, 0u);
            S_.key[lane] = ~0ull;
            S_.tri[lane] = kMiss;
            S_.rn[lane] = rn0;
        }
        if (RT_ROOT_VISIT && (!kTranslated || RT_XROOT_VISIT) && fast && !(P.root_ref & kLeafBit) && !(kCount && (P.debug & 32))) {
            // The root visit in the seed (round 6): every ray that enters the
            // root box visits the root's record, the same for every lane, so
            // its 64 B arrive through the scalar cache, and the pool starts
            // one level down (each ray's kept children, pushed with their
            // path codes by fast_slot as a popped root item would push them).
            // A chain-bound unit's pool chain shortens by a level; the visit
            // set and the counters are the reference's.
            float t0, t1;
            const bool has = root_pass<kCount>(P, R0, live, t0, t1, C.n_int, C.n_desc);
            __builtin_amdgcn_wave_barrier();  // (the rays' LDS fields are written)
            float4 q0, q1, q2, q3;
            root_record(P, q0, q1, q2, q3);
            const uint4 it = make_uint4(P.root_ref, __float_as_uint(t0), __float_as_uint(t1), ((uint32_t)lane << 26) | 1u);
            if constexpr (kTranslated)
                n = xfast_slot<RL::kStride, kCount, false, 0, 8, kOdP>(P, items, 0, S_.ray, S_.key, S_.tri, it, has, q0, q1,
                                                                     q2, q3, C.n_int, C.n_leaf, C.n_acc, C.n_desc);
            else
                n = fast_slot<RL::kStride, kCount, 8>(P, items, 0, S_.ray, S_.key, S_.tri, it, has, q0, q1, q2, q3,
                                                      C.n_int, C.n_leaf, C.n_acc, C.n_desc);
            __builtin_amdgcn_wave_barrier();
            // (counted as the pool iteration it replaces: the units' costs,
            // and so the cost order and its split thresholds, stay as before)
            iters = 1;
            popped = (uint32_t)__builtin_popcountll(__ballot(has));
        } else {
            n = seed_root<kCount>(P, items, R0, live, lane, C.n_int, C.n_desc);
            // diagnostics (debug bit 32, counting renders): stop after the root
            // test, so counter [4] is the number of pixels whose root test passes
            // (bench.py's roofline without the root-miss visits)
            if (kCount && (P.debug & 32)) n = 0;
        }
    }
    if (fast) {
        // one instance of the walk per octant (the views' rays look along +z
        // or -z; x and y change sign across the frame), the mixed one else;
        // untranslated walks take the kFast slots, translated ones xfast_slot
#define RT_OCT_WALK(o)                                                                                               \
    pool_walk<kCap, RL::kStride, kTranslated, kCount, false, 0, !kTranslated, o, kTranslated, kOdP>(                   \
        P, items, S_.ray, S_.key, S_.tri, n, lane, iters, popped, C.n_int, C.n_leaf, C.n_acc, C.n_desc)
        switch (oct) {
        case 0: RT_OCT_WALK(0); break;
        case 1: RT_OCT_WALK(1); break;
        case 2: RT_OCT_WALK(2); break;
        case 3: RT_OCT_WALK(3); break;
        case 4: RT_OCT_WALK(4); break;
        case 5: RT_OCT_WALK(5); break;
        case 6: RT_OCT_WALK(6); break;
        case 7: RT_OCT_WALK(7); break;
        default: RT_OCT_WALK(8); break;
        }
#undef RT_OCT_WALK
    }
    else
        pool_walk<kCap, RL::kStride, kTranslated, kCount, false, 0, false, 8, false, kOdP>(P, items, S_.ray, S_.key, S_.tri,
                                                                                       n, lane, iters, popped,
                                                            C.n_int, C.n_leaf, C.n_acc, C.n_desc);
    float cam[3];
    Ray R;
    {
        // the pixel is recomputed from the lane index behind an empty asm, so
        // neither the first ray's partial products nor the pixel's output
        // index stay live (and spilled) across the walk
        // (the rsqrt21 factor comes back from LDS: the same float, 21
        // Newton steps fewer)
        int32_t l2 = lane;
        asm volatile("" : "+v"(l2));
        live = unit_pixel(P, U, nrows, l2, px, ncols);
        float rn = lane < kRays ? S_.rn[lane] : 1.0f;
        camera_ray<true, !kTranslated>(P, px, live, cam, R, rn);
    }
    unsigned long long kbest = ~0ull;
    uint32_t best = kMiss;
    if (lane < kRays) {
        kbest = S_.key[lane];
        best = kbest == ~0ull ? kMiss : S_.tri[lane];
    }
    bool shadowed = false;
    if constexpr (kShadow > 0) {
        // the shadow segment of each hit: from the light to H = d*r - od
        const bool sh_live = live && best != kMiss;
        Ray Sh;
        Sh.odx = -2.0f; Sh.ody = -2.0f; Sh.odz = -2.0f;
        Sh.rx = 1.0f; Sh.ry = 1.0f; Sh.rz = 1.0f;
        float lmax = 0.0f;
        if (sh_live) {
            const float d = __uint_as_float((uint32_t)(kbest >> 32));
            float sx = ((d * R.rx) - R.odx) - 2;
            float sy = ((d * R.ry) - R.ody) - 2;
            float sz = ((d * R.rz) - R.odz) - 2;
            lmax = sqrtf((sx * sx) + (sy * sy) + (sz * sz)) * 0.9990234375f;  // correctly rounded sqrt
            const float r = rsqrt21(sx, sy, sz);
            Sh.rx = sx * r; Sh.ry = sy * r; Sh.rz = sz * r;
        }
        finish_ray(Sh);
        if (lane < kRays) {
            store_ray(&S_.ray[lane], RL::kStride, Sh, true, lmax, best);
            S_.key[lane] = ~0ull;
        }
        __builtin_amdgcn_wave_barrier();
        // the translated kFast slots when the light's proof holds
        // (rt_api.cpp fast_proof_shadow: the root box beyond the light's
        // plane on axis P.sh_axis) and every live shadow ray points into that
        // side with normal, nonzero components: then every box's entry
        // parameter is >= 2^-20 for it
        const float sk = P.sh_axis == 0 ? Sh.rx : P.sh_axis == 1 ? Sh.ry : Sh.rz;
        const bool sh_ok = fabsf(Sh.rx) >= 0x1p-126f && fabsf(Sh.ry) >= 0x1p-126f && fabsf(Sh.rz) >= 0x1p-126f &&
                           (P.sh_neg ? sk < 0.0f : sk > 0.0f);
        const bool sh_fast = P.fast_sh && __ballot(sh_live && !sh_ok) == 0ull;
        if (RT_ROOT_VISIT && sh_fast && !(P.root_ref & kLeafBit)) {
            // the root visit in the seed, as for the primary walk (every
            // shadow ray starts at the light)
            float t0, t1;
            const bool has = root_pass<kCount, true>(P, Sh, sh_live, t0, t1, C.n_int, C.n_desc, lmax);
            float4 q0, q1, q2, q3;
            root_record(P, q0, q1, q2, q3);
            const uint4 it = make_uint4(P.root_ref, __float_as_uint(t0), __float_as_uint(t1), ((uint32_t)lane << 26) | 1u);
            n = xfast_slot<RL::kStride, kCount, true, ((kShadow - 1) & 3), 8>(P, items, 0, S_.ray, S_.key, S_.tri, it, has,
                                                                             q0, q1, q2, q3, C.n_int, C.n_leaf, C.n_acc,
                                                                             C.n_desc);
            __builtin_amdgcn_wave_barrier();
            iters += 1;
            popped += (uint32_t)__builtin_popcountll(__ballot(has));
        } else {
            n = seed_root<kCount, true>(P, items, Sh, sh_live, lane, C.n_int, C.n_desc, lmax);
        }
        int sh_oct = 8;  // the octant every live shadow ray lies in (slab_pair_xoct), 8 = mixed
        if (RT_SH_OCT && sh_fast) {
            const unsigned long long LV = __ballot(sh_live), PX = __ballot(sh_live && Sh.rx > 0.0f),
                                     PY = __ballot(sh_live && Sh.ry > 0.0f), PZ = __ballot(sh_live && Sh.rz > 0.0f);
            if ((PX == 0ull || PX == LV) && (PY == 0ull || PY == LV) && (PZ == 0ull || PZ == LV))
                sh_oct = (PX == LV ? 1 : 0) | (PY == LV ? 2 : 0) | (PZ == LV ? 4 : 0);
        }
        if (sh_fast) {
#define RT_SH_WALK(o)                                                                                                \
    pool_walk<kCap, RL::kStride, true, kCount, true, kShadow - 1, false, o, true>(                                     \
        P, items, S_.ray, S_.key, S_.tri, n, lane, iters, popped, C.n_int, C.n_leaf, C.n_acc, C.n_desc)
            if (RT_SH_OCT) {
                switch (sh_oct) {
                case 0: RT_SH_WALK(0); break;
                case 1: RT_SH_WALK(1); break;
                case 2: RT_SH_WALK(2); break;
                case 3: RT_SH_WALK(3); break;
                case 4: RT_SH_WALK(4); break;
                case 5: RT_SH_WALK(5); break;
                case 6: RT_SH_WALK(6); break;
                case 7: RT_SH_WALK(7); break;
                default: RT_SH_WALK(8); break;
                }
            } else {
                RT_SH_WALK(8);
            }
#undef RT_SH_WALK
        } else
            pool_walk<kCap, RL::kStride, true, kCount, true, kShadow - 1>(P, items, S_.ray, S_.key, S_.tri, n, lane, iters,
                                                                         popped, C.n_int, C.n_leaf, C.n_acc, C.n_desc);
        if (lane < kRays) shadowed = S_.key[lane] == 0ull;
    }
    if (P.dbg && lane == 0 && dbg_slot != kNoDbg) {  // diagnostics: the unit's start/end clock (100 MHz) and pool iterations
        P.dbg[3 * dbg_slot] = t_start;
        P.dbg[3 * dbg_slot + 1] = __builtin_amdgcn_s_memrealtime();
        P.dbg[3 * dbg_slot + 2] = iters | ((unsigned long long)popped << 32);
    }
    // tile order 3: this unit's pool iterations (a split unit of half the
    // pixels reports twice its own: the tile's cost as a whole-tile unit, about)
    if (cost && lane == 0) *cost = iters * (uint32_t)(kRays / (nrows * ncols));
    __builtin_amdgcn_wave_barrier();  // LDS of this unit is read; the next unit may overwrite it
    if (!live) return;
    shade_out<kWriteHit, kCount>(P, px, R, cam, kbest, best, shadowed, C);
}

__device__ __forceinline__ void count_flush(const TraceParams& P, const Counts& C) {
    // every lane (also those past the frame edge) processed pool items;
    // counter [2] counts valid candidates here (>= the DFS's accept events)
    wave_count_add(&P.counters[0], C.n_int);
    wave_count_add(&P.counters[1], C.n_leaf);
    wave_count_add(&P.counters[2], C.n_acc);
    wave_count_add(&P.counters[3], C.n_hit);
    wave_count_add(&P.counters[4], C.n_desc);
}

// Root test of one coarse 8x8 group (all 64 lanes): returns the ballot of
// lanes whose root test passes; lanes whose kRays-pixel sub-tile has no
// passing ray write the background now.  The sub-tiles with a passing ray are
// traced by trace_unit, which repeats the same root test, so a coarse group's
// pixels are exactly what fine units would produce; only the packing of work
// into waves differs.
//
// A group first tries a cheap test (below: identity transform, then any
// transform): the ray normalised by the hardware rsqrt / rcp instead of the
// 21-step Newton loop and correctly rounded divisions.  Its slab parameters
// are within ~1e-6 (relative) of the exact ones, so a pixel whose test fails
// by a 1e-3 relative margin (or whose entry lies behind the eye by more than
// 1e-12) fails the exact test too; rays with a zero or tiny component, a NaN,
// or any doubt take the exact test.  When every pixel of the group is such a
// certain miss the group is background without the exact rays.
__device__ __forceinline__ bool root_certain_miss(const TraceParams& P, int32_t ix, int32_t iy) {
    // (float)ix of the reference's unsigned pixel index: exact and equal for any ix < 2^32
    const float fx = (float)(uint32_t)ix, fy = (float)(uint32_t)iy;
    const float x = P.n_mod[0] + P.u_mod[0] * fx + P.v_mod[0] * fy;
    const float y = P.n_mod[1] + P.u_mod[1] * fx + P.v_mod[1] * fy;
    const float z = P.n_mod[2] + P.u_mod[2] * fx + P.v_mod[2] * fy;
    const float r = __builtin_amdgcn_rsqf((x * x) + (y * y) + (z * z));
    const float dx = x * r, dy = y * r, dz = z * r;
    if (!(fabsf(dx) > 1e-6f && fabsf(dy) > 1e-6f && fabsf(dz) > 1e-6f)) return false;
    const float ix_ = __builtin_amdgcn_rcpf(dx), iy_ = __builtin_amdgcn_rcpf(dy), iz_ = __builtin_amdgcn_rcpf(dz);
    const float* b = P.root_box;
    const float t0x = (dx > 0 ? b[0] : b[1]) * ix_, t1x = (dx > 0 ? b[1] : b[0]) * ix_;
    const float t0y = (dy > 0 ? b[2] : b[3]) * iy_, t1y = (dy > 0 ? b[3] : b[2]) * iy_;
    const float t0z = (dz > 0 ? b[4] : b[5]) * iz_, t1z = (dz > 0 ? b[5] : b[4]) * iz_;
    const float maxt0 = fmaxf(t0z, fmaxf(t0x, t0y)), mint1 = fminf(t1z, fminf(t1x, t1y));
    if (!(fabsf(maxt0) < 1e30f && fabsf(mint1) < 1e30f)) return false;  // NaN or huge: exact test
    const float tol = 1e-3f * (fabsf(maxt0) + fabsf(mint1));
    return mint1 < maxt0 - tol || (maxt0 < -tol && maxt0 < -1e-12f);
}

// The same under an object transform (rotation rows X, offset od; the
// reference's ray R = X3 * cam, slab parameters t = (b + od) / R per axis,
// TD/Trixel.cu:60-95).  Bounds, per axis i, with S_i = sum_j |X_ij cam_j|:
//   * cam from the hardware rsq differs from the exact (21-step) ray by a
//     common factor within ~1.2e-6, and each path's dot product rounds by at
//     most 3 ulps of S_i, so |R_i(approx) - R_i(exact)| <= E_i = 4e-6 S_i;
//   * with |R_i| > 4e-3 S_i (rho_i = E_i / |R_i| < 1e-3, so both rays share
//     the sign and no component is near zero), b / R_i and od_i / R_i move by
//     at most 1.01 rho_i of their size, and the float roundings of either
//     path's t0 / t1 (rcp, products, sum) stay below 2e-6 of
//     M_i = (max |b| + |od_i|) / |R_i|;
//   * max / min move by at most the largest per-axis bound e.
// So exact maxt0, mint1 lie within e of these, and a miss by a margin of
// 2e + 1e-5 (|maxt0| + |mint1|) + 1e-12 is a miss of the exact double test
// (mint1 >= maxt0 - 1e-16 && maxt0 > -1e-16).  Any doubt: the exact test.
__device__ __forceinline__ bool root_certain_miss_xf(const TraceParams& P, int32_t ix, int32_t iy) {
    const float fx = (float)(uint32_t)ix, fy = (float)(uint32_t)iy;
    const float x = P.n_mod[0] + P.u_mod[0] * fx + P.v_mod[0] * fy;
    const float y = P.n_mod[1] + P.u_mod[1] * fx + P.v_mod[1] * fy;
    const float z = P.n_mod[2] + P.u_mod[2] * fx + P.v_mod[2] * fy;
    const float r = __builtin_amdgcn_rsqf((x * x) + (y * y) + (z * z));
    const float c0 = x * r, c1 = y * r, c2 = z * r;
    const float* X = P.xf;
    const float* b = P.root_box;
    float maxt0 = -INFINITY, mint1 = INFINITY, e = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float a0 = X[4 * i], a1 = X[4 * i + 1], a2 = X[4 * i + 2], od = X[4 * i + 3];
        const float ri = -1 * (a0 * -c0 + a1 * -c1 + a2 * -c2);
        const float si = fabsf(a0 * c0) + fabsf(a1 * c1) + fabsf(a2 * c2);
        if (!(fabsf(ri) > 4e-3f * si && si < 1e30f)) return false;
        const float inv = __builtin_amdgcn_rcpf(ri), o = od * inv;
        const float lo = b[2 * i], hi = b[2 * i + 1];
        const float t0 = (ri > 0 ? lo : hi) * inv + o, t1 = (ri > 0 ? hi : lo) * inv + o;
        const float rho = 4.01e-6f * si * fabsf(inv);  // rcp within an ulp of 1 / ri: no divide
        const float m = (fmaxf(fabsf(lo), fabsf(hi)) + fabsf(od)) * fabsf(inv);
        maxt0 = fmaxf(maxt0, t0);
        mint1 = fminf(mint1, t1);
        e = fmaxf(e, m * (1.01f * rho + 2e-6f));
    }
    if (!(fabsf(maxt0) < 1e30f && fabsf(mint1) < 1e30f && e < 1e30f)) return false;  // NaN or huge: exact test
    // 2e is the bound; the relative 1e-5 is a safety factor over its 2e-6
    // rounding allowance (1e-3, the identity test's margin, left the ring of
    // groups next to the fine tiles to the exact test: 18.7 us per kernel)
    const float tol = 2.0f * e + 1e-5f * (fabsf(maxt0) + fabsf(mint1)) + 1e-12f;
    return mint1 < maxt0 - tol || maxt0 < -tol;
}

// A whole 8x8 group at once (RT_GROUP_MISS): the unnormalised direction
// D = X3 (n_mod + u_mod fx + v_mod fy) is affine in the pixel, so over the
// group each D_i lies between its values at the four corners; widened by
// e_i = 1e-5 sum_j |X_ij| (|n_j| + |u_j| fx_max + |v_j| fy_max) it holds
// every pixel's float ray divided by its (positive) norm -- the float
// evaluation of c, the 21-step normalisation and the rotation stay within a
// few ulps of that sum.  An axis whose interval touches 0 leaves the group to
// the per-pixel tests (0/0 = NaN drops an axis in the reference).  With the
// signs fixed, t0_i = (near_i + od_i) / D_i and t1_i = (far_i + od_i) / D_i
// are monotone in D_i, so every pixel's maxt0 >= L0 = max_i min t0_i and
// mint1 <= U1 = min_i max t1_i (in the unnormalised scale; the reference's t
// are these times the norm, a common positive factor, plus float rounding of
// at most a few ulps of M = (|near| + |far| + |od|) / |D|).  A margin of
// 1e-4 M_max + 1e-3 (|L0| + |U1|) + 1e-12 above that rounding makes
// L0 > U1 + margin a miss of every pixel's exact test (mint1 < maxt0 -
// 1e-16), and U1 < -margin one too (maxt0 <= mint1 + 1e-16 < 0); so is
// U0 < -margin with U0 = max_i max t0_i >= every pixel's maxt0 (an eye
// inside the root box, round 6: every entry lies behind it).
__device__ __forceinline__ bool group_certain_miss(const TraceParams& P, const Unit& G) {
    const int32_t y0 = (P.rank + G.slot * P.nranks) * kTileH + G.yin;
    const float fx0 = (float)(uint32_t)G.x0, fx1 = (float)(uint32_t)(G.x0 + 7);
    const float fy0 = (float)(uint32_t)y0, fy1 = (float)(uint32_t)(y0 + 7);
    const float* X = P.xf;
    const float* b = P.root_box;
    float L0 = -INFINITY, U1 = INFINITY, U0 = -INFINITY, mmax = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float x0 = X[4 * i], x1 = X[4 * i + 1], x2 = X[4 * i + 2], od = X[4 * i + 3];
        const float A = x0 * P.n_mod[0] + x1 * P.n_mod[1] + x2 * P.n_mod[2];
        const float B = x0 * P.u_mod[0] + x1 * P.u_mod[1] + x2 * P.u_mod[2];
        const float Cc = x0 * P.v_mod[0] + x1 * P.v_mod[1] + x2 * P.v_mod[2];
        const float e = 1e-5f * (fabsf(x0) * (fabsf(P.n_mod[0]) + fabsf(P.u_mod[0]) * fx1 + fabsf(P.v_mod[0]) * fy1) +
                                 fabsf(x1) * (fabsf(P.n_mod[1]) + fabsf(P.u_mod[1]) * fx1 + fabsf(P.v_mod[1]) * fy1) +
                                 fabsf(x2) * (fabsf(P.n_mod[2]) + fabsf(P.u_mod[2]) * fx1 + fabsf(P.v_mod[2]) * fy1));
        const float d00 = A + B * fx0 + Cc * fy0, d01 = A + B * fx0 + Cc * fy1;
        const float d10 = A + B * fx1 + Cc * fy0, d11 = A + B * fx1 + Cc * fy1;
        const float dlo = fminf(fminf(d00, d01), fminf(d10, d11)) - e;
        const float dhi = fmaxf(fmaxf(d00, d01), fmaxf(d10, d11)) + e;
        if (!(dlo > 0.0f || dhi < 0.0f)) return false;  // touches 0 (or NaN): the per-pixel tests
        const bool pos = dlo > 0.0f;
        const float lo = b[2 * i], hi = b[2 * i + 1];
        const float n0 = (pos ? lo : hi) + od, n1 = (pos ? hi : lo) + od;
        // t = n / D over D in [dlo, dhi] (one sign): extremes at the ends
        const float a0 = n0 / dlo, a1 = n0 / dhi, c0 = n1 / dlo, c1 = n1 / dhi;
        L0 = fmaxf(L0, fminf(a0, a1));
        U0 = fmaxf(U0, fmaxf(a0, a1));
        U1 = fminf(U1, fmaxf(c0, c1));
        mmax = fmaxf(mmax, (fabsf(lo) + fabsf(hi) + fabsf(od)) / fminf(fabsf(dlo), fabsf(dhi)));
    }
    if (!(fabsf(L0) < 1e30f && fabsf(U1) < 1e30f && fabsf(U0) < 1e30f && mmax < 1e30f)) return false;
    const float margin = 1e-4f * mmax + 1e-3f * (fabsf(L0) + fabsf(U1) + fabsf(U0)) + 1e-12f;
    return L0 > U1 + margin || U1 < -margin || U0 < -margin;
}

//
#ifndef RT_GROUP_MISS
#define RT_GROUP_MISS 1
#endif
// Groups at least 2 pixels outside the root box's screen rectangle
// (P.far_rect, identity transform only) skip even that: the rectangle is the
// box's exact projection (in double, from the same float basis), a pixel's
// float ray deviates from its exact direction by ~1e-6 rad against the
// ~1e-3 rad of two pixels, and with a zero object offset the slab parameters
// are single roundings of bound / D, so the test fails -- unless a component
// of the ray is zero (0/0 = NaN drops that axis from the test) or tiny,
// which each pixel checks.
__device__ __forceinline__ bool far_group(const TraceParams& P, const Unit& G) {
    const int32_t y0 = (P.rank + G.slot * P.nranks) * kTileH;
    return G.x0 + 7 < P.far_rect[0] || G.x0 > P.far_rect[1] || y0 + 7 < P.far_rect[2] || y0 > P.far_rect[3];
}

__device__ __forceinline__ bool ray_has_tiny_component(const TraceParams& P, int32_t ix, int32_t iy) {
    const float fx = (float)(uint32_t)ix, fy = (float)(uint32_t)iy;
    const float x = P.n_mod[0] + P.u_mod[0] * fx + P.v_mod[0] * fy;
    const float y = P.n_mod[1] + P.u_mod[1] * fx + P.v_mod[1] * fy;
    const float z = P.n_mod[2] + P.u_mod[2] * fx + P.v_mod[2] * fy;
    return !(fabsf(x) > 1e-30f && fabsf(y) > 1e-30f && fabsf(z) > 1e-30f);
}

// A far group (see above) whose rays have no tiny component is background:
// writes it and returns true; otherwise returns false and writes nothing.
template <bool kWriteHit, bool kCount>
__device__ __forceinline__ bool fill_far(const TraceParams& P, const Unit& G, int lane, Counts& C) {
    // P.far_all: the host proved the box behind the eye for every pixel
    // (rt_api.cpp box_behind, any transform, zero components included)
    if (!P.far_all && !far_group(P, G)) return false;
    Pixel px;
    const bool live = unit_pixel(P, G, 8, lane, px);
    if (!P.far_all && __ballot(live && ray_has_tiny_component(P, px.x, px.y)) != 0ull) return false;
    if (live) {
        put_pixel(P, px.out, kBackground, false);
        if (kWriteHit) P.hit[px.out] = (int64_t)-1;
        if (kCount) C.n_int += 1u;  // the root visit, which fails
    }
    return true;
}

// A group known to miss: every pixel background (the root visit fails).
template <bool kWriteHit, bool kCount>
__device__ __forceinline__ void fill_background(const TraceParams& P, const Unit& G, int lane, Counts& C) {
    Pixel px;
    if (unit_pixel(P, G, 8, lane, px)) {
        put_pixel(P, px.out, kBackground, false);
        if (kWriteHit) P.hit[px.out] = (int64_t)-1;
        if (kCount) C.n_int += 1u;  // the root visit, which fails
    }
}

// A coarse group every pixel of which is a certain miss (above) is
// background: writes it and returns true; otherwise writes nothing.
template <bool kWriteHit, bool kCount>
__device__ __forceinline__ bool coarse_sure(const TraceParams& P, const Unit& G, int lane, Counts& C) {
    Pixel px;
    const bool live = unit_pixel(P, G, 8, lane, px);
    const bool sure = !live || (P.plain_xf ? root_certain_miss(P, px.x, px.y) : root_certain_miss_xf(P, px.x, px.y));
    if (__ballot(!sure) != 0ull) return false;
    if (live) {
        put_pixel(P, px.out, kBackground, false);
        if (kWriteHit) P.hit[px.out] = (int64_t)-1;
        if (kCount) C.n_int += 1u;  // the root visit, which fails
    }
    return true;
}

// The exact root test of a coarse group (after coarse_sure, when it applies).
template <int kRays, bool kWriteHit, bool kCount>
__device__ __forceinline__ unsigned long long coarse_root(const TraceParams& P, const Unit& G, int lane, Counts& C) {
    Pixel px;
    const bool live = unit_pixel(P, G, 8, lane, px);
    float cam[3], t0, t1;
    Ray R;
    camera_ray(P, px, live, cam, R);
    uint32_t ni = 0, nd = 0;
    const bool has = root_pass<kCount>(P, R, live, t0, t1, ni, nd);
    const unsigned long long b = __ballot(has);
    constexpr unsigned long long kSub = (1ull << kRays) - 1;
    const bool traced = ((b >> ((lane / kRays) * kRays)) & kSub) != 0;
    if (live && !traced) {
        put_pixel(P, px.out, kBackground, false);
        if (kWriteHit) P.hit[px.out] = (int64_t)-1;
        if (kCount) C.n_int += ni;  // the root visit; no root test passed in this sub-tile
    }
    return b;
}

// kShadow: a second pool walk traces one shadow ray per hit (SURVEY.md §8a
// a12; definition in oracle/oracle.c trace_shadow): the segment from the light
// (2,2,2) to the hit, walked from the light with the reference's rules and
// entering only the boxes the segment enters (entry parameter below Lmax).
// One fine tile per block (the tiles covering the root box's screen
// rectangle, or the whole frame), one unit per wave.
// Occupancy: a 16-ray block's LDS (26 KB) admits 6 blocks per CU, and
// __launch_bounds__ for 6 waves per SIMD caps the registers at 80 (round 2:
// dragon 1080p 13.7k -> 14.7k FPS with two frames in flight, the 93 % fill
// view 940 -> 873 us per frame).  On the round-5/6 kernels the timed 16-ray
// instances fit 80 VGPRs without scratch; only the counting instances (kCount,
// untimed) spill, and the shadow instances (84 VGPRs) run 5 waves per SIMD.
// profiles/r06/kernel_resources.txt (tools/kernel_resources.py over the built
// library) lists every instance's VGPRs, scratch and waves per SIMD.
#ifndef RT_KD3_OCC
#define RT_KD3_OCC 6
#endif
#define RT_KD3_BOUNDS(threads) __launch_bounds__(threads, RT_KD3_OCC)
// One block of k_trace_kd3's grid: block index b (blockIdx.x, or the virtual
// index within a multi-frame launch, below).
template <int kRays, bool kTranslated, bool kWriteHit, bool kCount, int kShadow, int kCap, int kRayVec>
__device__ __forceinline__ void kd3_block(const TraceParams& P, WaveLds<kRays, kCap, kRayVec>* s_lds, int32_t b,
                                          int wv, int lane) {
    constexpr int kWaves = kd3_waves(kRays);
    Counts C;
    const int32_t ntiles = P.tiles_x * P.block_rows;
    const int32_t bslot = b;  // diagnostics slot of this block
    // a multi-frame launch's padding blocks (XCD-mapped tile orders)
    if (b >= ntiles + P.split + P.fill_blocks) return;
    // blocks: 2 per split tile, 1 per other fine tile, then the far fill
    if (b >= ntiles + P.split) {
        // fused far fill: blocks after the fine tiles write the coarse groups,
        // all far by construction (set_fine_region); unrolled as in k_coarse_kd3
        const int32_t j0 = ((b - ntiles - P.split) * kWaves + wv) * P.coarse_per_wave;
        const int32_t j1 = min(j0 + P.coarse_per_wave, (int32_t)P.coarse_groups);
        bool ok = true;
#pragma unroll 8
        for (int g = 0; g < kCoarseMax; g++) {
            const int32_t j = j0 + g;
            if (j < j1) ok = fill_far<kWriteHit, kCount>(P, coarse_unit(P, j), lane, C) && ok;
        }
        if (!ok && lane == 0) atomicOr(P.err, 4);  // a group the host promised far was not
        if (kCount) count_flush(P, C);
        return;
    }
    // Split tiles (tile order 3; the host names the heaviest P.split tiles of
    // its cost order, order[0..split)): blocks 2k and 2k + 1 render the halves
    // of tile order[k] -- with 16-ray units one 8-pixel row per wave, with
    // 8-ray units a 4-pixel half row per wave -- which halves the heaviest
    // units' pool chains; the other tiles follow.  (Quarters of the heaviest
    // tiles, four 4-ray units of a 16-ray unit, measured slower: dragon
    // 960x540 43.0-45.8k -> 38.0-39.4k FPS, r03s; block-cooperative units, a
    // whole block on one pool, slower at every threshold, r04.)
    const bool split = b < 2 * P.split;
    const int32_t ti = split ? P.order[b >> 1] : tile_index(P, b - P.split);
    if ((uint32_t)ti >= (uint32_t)ntiles) {  // a stale order: never index past the grid
        if (lane == 0) atomicOr(P.err, 8);
        return;
    }
    uint32_t* cost = P.cost ? P.cost + kCostSlots * (size_t)ti + wv + (split ? (b & 1) * 4 : 0) : nullptr;
    if (cost && !split && lane == 0) cost[4] = 0u;  // no second half
    Unit U = unit_of_tile(P, ti, wv);
    if (split && kRays == 16) U.yin = (U.yin - wv * (kRays / 8)) + (b & 1) * kWaves + wv;
    if (split && kRays == 8) U.x0 += (b & 1) * 4;
    trace_unit<kRays, kCap, kRayVec, kTranslated, kWriteHit, kCount, kShadow>(
        P, s_lds[wv], U, lane, (size_t)bslot * kWaves + wv, cost, C, split && kRays == 16 ? 1 : kRays / 8,
        split && kRays == 8 ? 4 : 8);
    if (kCount) count_flush(P, C);
}

// Kernel 3: one frame, one block per grid slot.  A multi-frame launch
// (rt_run_frames with RT_LOOP_MULTIFRAME; P.pf_frames > 0) has pf_frames x
// pf_blocks blocks, frame-major: block i renders block i % pf_blocks of frame
// i / pf_blocks into P.pf_argb[(P.pf_seq0 + frame) % P.pf_nbuf].  Blocks are
// dispatched in index order, so frame f + 1's heaviest tiles start on the CUs
// frame f's tail frees, with no launch between frames (static scenes: every
// frame is the same frame).  (Interleaving the blocks of groups of 2-3
// frames measured the same, r04m-n.)
template <int kRays, bool kTranslated, bool kWriteHit, bool kCount, int kShadow>
__global__ RT_KD3_BOUNDS(64 * kd3_waves(kRays)) void k_trace_kd3(TraceParams P) {
    constexpr int kCap = pool_cap_for<kRays>();
    // float4s of per-ray data in LDS: translated primary walks read the
    // offset from the transform (kOdP), shadow walks keep Lmax and the hit
    constexpr int kRayVec = kShadow ? 5 : 3;
    __shared__ WaveLds<kRays, kCap, kRayVec> s_lds[kd3_waves(kRays)];
    const int wv = wave_id(), lane = (int)threadIdx.x & 63;
    int32_t b = (int32_t)blockIdx.x;
    if (P.pf_frames > 0) {
        const int32_t f = b / P.pf_blocks;
        b -= f * P.pf_blocks;
        // every wave's lane 0 stores the same pointer, then its own lanes read it
        if (lane == 0) s_pf_argb = P.pf_argb[(P.pf_seq0 + f) % P.pf_nbuf];
        __builtin_amdgcn_wave_barrier();
    }
    kd3_block<kRays, kTranslated, kWriteHit, kCount, kShadow, kCap, kRayVec>(P, s_lds, b, wv, lane);
}

// The coarse groups (every 8x8 group of this rank outside the fine tiles),
// P.coarse_per_wave (<= kCoarseMax) per wave.  A separate kernel: looping trace_unit inside
// the fine kernel costs it a third of its occupancy (80 -> 113 VGPRs).
template <int kRays, bool kTranslated, bool kWriteHit, bool kCount, int kShadow>
__global__ __launch_bounds__(128) void k_coarse_kd3(TraceParams P) {
    constexpr int kWaves = 2;
    constexpr int kCap = pool_cap_for<kRays>();
    constexpr int kRayVec = kShadow ? 5 : 3;
    constexpr unsigned long long kSub = (1ull << kRays) - 1;
    __shared__ WaveLds<kRays, kCap, kRayVec> s_lds[kWaves];
    const int wv = wave_id(), lane = (int)threadIdx.x & 63;
    Counts C;
    const unsigned long long t_start = P.dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const int32_t cw = (int32_t)blockIdx.x * kWaves + wv;
    const int32_t j0 = cw * P.coarse_per_wave;
    const int32_t j1 = min(j0 + P.coarse_per_wave, (int32_t)P.coarse_groups);
    // Far groups first, unrolled so their short independent chains overlap
    // (one after another they cost ~1 us each in latency); the rest after.
    const bool far_ok = P.plain_xf && !(P.root_ref & kLeafBit) && !(P.debug & 1);
    uint32_t pending = 0;
#pragma unroll 8
    for (int g = 0; g < kCoarseMax; g++) {
        const int32_t j = j0 + g;
        if (j < j1 && !(far_ok && fill_far<kWriteHit, kCount>(P, coarse_unit(P, j), lane, C))) pending |= 1u << g;
    }
    // the whole-group certain-miss test, one group per lane (RT_GROUP_MISS)
    if (RT_GROUP_MISS && !(P.root_ref & kLeafBit) && !(P.debug & 1)) {
        const int32_t jg = j0 + lane;
        const bool sure = lane < kCoarseMax && jg < j1 && ((pending >> lane) & 1u) &&
                          group_certain_miss(P, coarse_unit(P, jg));
        const uint32_t sure_mask = (uint32_t)__ballot(sure);
#pragma unroll 8
        for (int g = 0; g < kCoarseMax; g++)
            if ((sure_mask >> g) & 1u) fill_background<kWriteHit, kCount>(P, coarse_unit(P, j0 + g), lane, C);
        pending &= ~sure_mask;
    }
    // then the per-pixel certain-miss test of the rest, unrolled the same way
    // (one group after another, its rsq / rcp chains cost ~1 us each); the
    // groups left take the exact root test
    if (!(P.root_ref & kLeafBit) && !(P.debug & 1)) {
#pragma unroll 8
        for (int g = 0; g < kCoarseMax; g++)
            if (((pending >> g) & 1u) && coarse_sure<kWriteHit, kCount>(P, coarse_unit(P, j0 + g), lane, C))
                pending &= ~(1u << g);
    }
    while (pending) {
        const int32_t j = j0 + __builtin_ctz(pending);
        pending &= pending - 1;
        const Unit G = coarse_unit(P, j);
        const unsigned long long gmask = coarse_root<kRays, kWriteHit, kCount>(P, G, lane, C);
        for (int k = 0; k < 64 / kRays; k++)
            if ((gmask >> (k * kRays)) & kSub)
                trace_unit<kRays, kCap, kRayVec, kTranslated, kWriteHit, kCount, kShadow>(
                    P, s_lds[wv], Unit{G.x0, G.slot, k * (kRays / 8)}, lane, kNoDbg, nullptr, C);
    }
    if (P.dbg && lane == 0) {  // after the fine kernel's slots
        const size_t slot = (size_t)(P.tiles_x * P.block_rows + blockIdx.x) * kWaves + wv;
        P.dbg[3 * slot] = t_start;
        P.dbg[3 * slot + 1] = __builtin_amdgcn_s_memrealtime();
        P.dbg[3 * slot + 2] = 0xFFFFFFFFull;  // marks a coarse wave
    }
    if (kCount) count_flush(P, C);
}

// -------------------------------------------------------------- flat trace

// intersect_trixel_cuda (TD/Trixel.cu:173-209) fused with the shading.  The
// triangle loop index is wave-uniform, so the pair layout's records arrive
// through the scalar data cache into SGPRs; a screen on the signed layout
// (k_pair_tri) skips the correctly rounded division for the (common) rays
// that cannot pass u >= eps, v >= eps or w >= eps.
//
// The rest of one flat test (TD/Trixel.cu:185-205) for a ray that passed
// the screen: strict w < d, so among equal w the lowest index wins.
__device__ __forceinline__ void flat_accept(float f, float U, float V, float W, uint32_t t, float& d,
                                            uint32_t& best, uint32_t& n_acc) {
    if (!(f < kEpsF && f > -kEpsF)) {
        const float pe1 = 1.0f / f;   // == (float)(1.0 / (double)f)
        const float u = pe1 * U;
        const float v = pe1 * V;
        const float w = pe1 * W;
        if ((w < d) && !((u < kEpsF) || (v < kEpsF) || ((u + v) > 1.0f) || (w < kEpsF))) {
            d = w;
            best = t;
            n_acc++;
        }
    }
}

// One pair of the flat kernel's pair layout in registers (SGPRs: the loop
// index is wave-uniform) and its two tests as packed float2 arithmetic.
struct FlatPair {
    f2v e1x, e1y, e1z, e2x, e2y, e2z, tx, ty, tz, dqx, dqy, dqz, dw;
    __device__ __forceinline__ void load(const f2v* q) {
        e1x = q[0]; e1y = q[1]; e1z = q[2]; e2x = q[3]; e2y = q[4]; e2z = q[5];
        tx = q[6]; ty = q[7]; tz = q[8]; dqx = q[9]; dqy = q[10]; dqz = q[11]; dw = q[12];
    }
    // Loads pair `pair` of Q only after `prev`'s values have arrived: the
    // index is made to depend on one of them through `zero`, a run-time 0
    // the compiler cannot fold (an asm barrier would make the loads vector
    // loads), so waiting for prev never waits for this pair's loads.
    __device__ __forceinline__ void load_after(const f2v* __restrict__ Q, uint32_t pair, const FlatPair& prev,
                                               uint32_t zero) {
        pair ^= __float_as_uint(prev.dw.y) & zero;
        load(Q + 16 * (size_t)pair);
    }
    // The test, V first.  On the signed layout a triangle can be accepted
    // only where f > 0, U > 0 and V > 0 (or NaN): min3 ignores NaN, so a NaN
    // U or V never rejects by itself, and a NaN f fails the full test.  v's
    // numerator V = r . d_q depends on the ray only through one dot product; V <= 0 in every lane of the wave for both triangles --
    // an 8x8 pixel tile wholly on the outer side of the two edge planes,
    // about half the (tile, pair) combinations -- skips the cross product,
    // f and U (19 of the pair's 24 packed operations); triangle t then t + 1,
    // so equal w keeps the lower index.
    __device__ __forceinline__ void test_signed_v(const f2v X, const f2v Y, const f2v Z, uint32_t t, float& d,
                                                  uint32_t& best, uint32_t& n_acc) const {
        const f2v V = (X * dqx + Y * dqy) + Z * dqz;
        if (!(V.x <= 0.0f) || !(V.y <= 0.0f)) {
            const f2v qx = Y * e2z - Z * e2y;
            const f2v qy = Z * e2x - X * e2z;
            const f2v qz = X * e2y - Y * e2x;
            const f2v f = (qx * e1x + qy * e1y) + qz * e1z;
            const f2v U = (qx * tx + qy * ty) + qz * tz;
            const float m0 = fminf(fminf(U.x, V.x), f.x), m1 = fminf(fminf(U.y, V.y), f.y);
            if (!(fmaxf(m0, m1) <= 0.0f)) {
                if (!(m0 <= 0.0f)) flat_accept(f.x, U.x, V.x, dw.x, t, d, best, n_acc);
                if (!(m1 <= 0.0f)) flat_accept(f.y, U.y, V.y, dw.y, t + 1, d, best, n_acc);
            }
        }
    }
};

// Phong of a flat-list pixel (TD/Camera.cu:19-69) from its nearest hit
// (w = d, triangle best), or the background; writes the pixel (and hit).
template <bool kWriteHit>
__device__ __forceinline__ void flat_shade_out(const TraceParams& P, const Pixel& px, const float rmd[3], float d,
                                               uint32_t best) {
    uint32_t argb = kBackground;
    if (best != kMiss) {
        const float4 N = P.shade[2 * (size_t)best];
        const float4 M = P.shade[2 * (size_t)best + 1];
        const float pnt[3] = {d * rmd[0], d * rmd[1], d * rmd[2]};
        const float nrm[3] = {N.x, N.y, N.z};
        const float rad[3] = {M.x, M.y, M.z};
        argb = phong(pnt, nrm, rmd, rad);
    }
    put_pixel(P, px.out, argb, best != kMiss);
    if (kWriteHit) P.hit[px.out] = best == kMiss ? (int64_t)-1 : (int64_t)best;
}

// The flat list in one pass (RT_OPT_FLAT 9; counting renders): pair p + 1's
// scalar loads are issued once pair p's have arrived (scalar loads return
// out of order, so a wait is always for all of them) and overlap pair p's
// tests.  Forms 0-8 of rounds 1-2 (one triangle per iteration, unpacked
// pairs, packed pairs without the signed layout or the V-first skip)
// measured 19.8-35.0 ms per C2 frame against this form's 18.3.
template <bool kWriteHit, bool kCount>
__global__ __launch_bounds__(kTileWFlat * kTileH) void k_trace_flat(TraceParams P) {
    Pixel px;
    if (!pixel_of_thread(P, px)) return;
    float rmd[3];
    primary_ray(P, px.x, px.y, rmd);
    float d = kDrawDistance;
    uint32_t best = kMiss;
    uint32_t n_acc = 0;
    const uint32_t ntri = P.ntri;
    // pair p = triangles (2p, 2p+1): 13 float2 (e1, e2, d_t, d_q, d_w), 128 B;
    // an odd count's last pair holds a dead twin (d_w = 0: never accepted)
    const f2v* __restrict__ Q = reinterpret_cast<const f2v*>(P.tpair);
    const f2v X = {rmd[0], rmd[0]}, Y = {rmd[1], rmd[1]}, Z = {rmd[2], rmd[2]};
    const uint32_t npair = (ntri + 1) >> 1;
    const uint32_t zero = ntri >> 31;  // 0: scenes hold < 2^29 triangles
    FlatPair a, b;
    a.load(Q);
    uint32_t p = 0;
    for (; p + 1 < npair; p += 2) {
        b.load_after(Q, p + 1, a, zero);
        a.test_signed_v(X, Y, Z, 2 * p, d, best, n_acc);
        a.load_after(Q, min(p + 2, npair - 1), b, zero);
        b.test_signed_v(X, Y, Z, 2 * p + 2, d, best, n_acc);
    }
    if (p < npair) a.test_signed_v(X, Y, Z, 2 * p, d, best, n_acc);
    flat_shade_out<kWriteHit>(P, px, rmd, d, best);
    if (kCount) {
        wave_count_add(&P.counters[1], ntri);
        wave_count_add(&P.counters[2], n_acc);
        wave_count_add(&P.counters[3], best != kMiss ? 1u : 0u);
    }
}

// Chunked flat list (RT_OPT_FLAT 12, the default; renders without counters): block b of a
// grid of fine blocks x P.flat_chunks tests its tile's rays against chunk
// b / fine of the pair list (k_trace_flat's loop: V first, pipelined loads) and
// folds each ray's nearest hit into P.flat_key[pixel] as the 64-bit minimum
// of (w bits, triangle); k_flat_shade then shades every pixel from its key
// and resets it.  w >= eps > 0, so the float bits order as the values, and
// the minimum over chunks of each chunk's first nearest triangle is the
// reference's first nearest triangle: the lowest index among equal w.  A
// chunk is an eighth (a quarter, a sixteenth) of a wave's work, so the grid
// runs in several rounds of short waves instead of one round of long ones.
__global__ __launch_bounds__(kTileWFlat * kTileH) void k_flat_chunk(TraceParams P) {
    const int32_t fine = P.tiles_x * P.block_rows;
    const int32_t chunk = (int32_t)blockIdx.x / fine, tb = (int32_t)blockIdx.x - chunk * fine;
    Pixel px;
    if (!pixel_of(P, tb, wave_id(), px)) return;
    float rmd[3];
    primary_ray(P, px.x, px.y, rmd);
    const f2v X = {rmd[0], rmd[0]}, Y = {rmd[1], rmd[1]}, Z = {rmd[2], rmd[2]};
    const f2v* __restrict__ Q = reinterpret_cast<const f2v*>(P.tpair);
    const uint32_t npair = (P.ntri + 1) >> 1;
    const uint32_t p0 = (uint32_t)(((uint64_t)chunk * npair) / (uint32_t)P.flat_chunks);
    const uint32_t p1 = (uint32_t)(((uint64_t)(chunk + 1) * npair) / (uint32_t)P.flat_chunks);
    if (p0 >= p1) return;
    float d = kDrawDistance;
    uint32_t best = kMiss, n_acc = 0;
    const uint32_t zero = P.ntri >> 31;  // 0: scenes hold < 2^29 triangles
    FlatPair a, b;
    a.load(Q + 16 * (size_t)p0);
    uint32_t p = p0;
    for (; p + 1 < p1; p += 2) {
        b.load_after(Q, p + 1, a, zero);
        a.test_signed_v(X, Y, Z, 2 * p, d, best, n_acc);
        a.load_after(Q, min(p + 2, p1 - 1), b, zero);
        b.test_signed_v(X, Y, Z, 2 * p + 2, d, best, n_acc);
    }
    if (p < p1) a.test_signed_v(X, Y, Z, 2 * p, d, best, n_acc);
    if (best != kMiss) atomicMin(&P.flat_key[px.out], ((unsigned long long)__float_as_uint(d) << 32) | best);
}

template <bool kWriteHit>
__global__ __launch_bounds__(kTileWFlat * kTileH) void k_flat_shade(TraceParams P) {
    Pixel px;
    if (!pixel_of_thread(P, px)) return;
    const unsigned long long key = P.flat_key[px.out];
    P.flat_key[px.out] = ~0ull;  // ready for the next frame on this stream
    float rmd[3];
    primary_ray(P, px.x, px.y, rmd);
    const bool hit = key != ~0ull;
    flat_shade_out<kWriteHit>(P, px, rmd, hit ? __uint_as_float((uint32_t)(key >> 32)) : kDrawDistance,
                              hit ? (uint32_t)key : kMiss);
}

// The flat kernel's pair layout: pair p <- camera-relative records 2p, 2p+1,
// each field as (value of 2p, value of 2p+1); a missing twin is dead (all
// zero: d_w = 0 fails the screen, and its full test gives w = 0 < eps).
//
// Signed: a triangle with d_w < 0 is stored with e1, d_t and d_q negated and
// d_w = |d_w|.  Negation is exact and commutes with every rounded product and
// sum, so the kernel's f, U, V come out exactly negated and u = U/f, v, w =
// d_w/f are unchanged bit for bit; only signs move, so that a triangle can be
// accepted only where f > 0 (w = d_w/f >= eps needs sign f = sign d_w).  A
// triangle with d_w = +-0 or NaN can never be accepted (w = 0 < eps, or
// w < d false): its e1 is stored as zero, so f = 0 and every form rejects it.
__global__ void k_pair_tri(const float4* __restrict__ trec, uint32_t ntri, float4* __restrict__ tpair) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t npair = (ntri + 1) >> 1;
    if (p >= npair) return;
    float a[13], b[13];
    const uint32_t t0 = 2 * p, t1 = 2 * p + 1;
    const float4* r0 = trec + 4 * (size_t)t0;
    const float4 A0 = r0[0], B0 = r0[1], C0 = r0[2], D0 = r0[3];
    a[0] = A0.x; a[1] = A0.y; a[2] = A0.z; a[3] = A0.w; a[4] = B0.x; a[5] = B0.y; a[6] = B0.z; a[7] = B0.w;
    a[8] = C0.x; a[9] = C0.y; a[10] = C0.z; a[11] = C0.w; a[12] = D0.x;
    for (int k = 0; k < 13; k++) b[k] = 0.0f;
    if (t1 < ntri) {
        const float4* r1 = trec + 4 * (size_t)t1;
        const float4 A1 = r1[0], B1 = r1[1], C1 = r1[2], D1 = r1[3];
        b[0] = A1.x; b[1] = A1.y; b[2] = A1.z; b[3] = A1.w; b[4] = B1.x; b[5] = B1.y; b[6] = B1.z; b[7] = B1.w;
        b[8] = C1.x; b[9] = C1.y; b[10] = C1.z; b[11] = C1.w; b[12] = D1.x;
    }
    for (int j = 0; j < 2; j++) {
        float* r = j ? b : a;
        const float dw = r[12];
        if (!(dw > 0.0f)) {
            // e1: 0-2, e2: 3-5 (kept), d_t: 6-8, d_q: 9-11 (k_cam_tri's order)
            const bool dead = !(dw < 0.0f);
            for (int k = 0; k < 12; k++)
                if (k < 3 || k >= 6) r[k] = (dead && k < 3) ? 0.0f : -r[k];
            r[12] = dead ? 0.0f : -dw;
        }
    }
    // field order of the kernel: e1 (3), e2 (3), d_t (3), d_q (3), d_w
    float4* o = tpair + 8 * (size_t)p;
    o[0] = make_float4(a[0], b[0], a[1], b[1]);
    o[1] = make_float4(a[2], b[2], a[3], b[3]);
    o[2] = make_float4(a[4], b[4], a[5], b[5]);
    o[3] = make_float4(a[6], b[6], a[7], b[7]);
    o[4] = make_float4(a[8], b[8], a[9], b[9]);
    o[5] = make_float4(a[10], b[10], a[11], b[11]);
    o[6] = make_float4(a[12], b[12], 0.0f, 0.0f);
    o[7] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// ------------------------------------------------------------------ prep

// init_tri_mem_cuda, TD/Trixel.cu:11-27, plus the Color::rad copy.
// tri_world = (p1.xyz, e1.x) (e1.yz, e2.xy) (e2.z, n.xyz); shade = (n, 0) (rad, 0)
__global__ void k_tri_world(const float* __restrict__ pts, const float* __restrict__ rad,
                            uint32_t ntri, float4* __restrict__ tw, float4* __restrict__ shade) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntri) return;
    const float* P = pts + 9 * (size_t)i;
    const float e1x = P[3] - P[0], e1y = P[4] - P[1], e1z = P[5] - P[2];
    const float e2x = P[6] - P[0], e2y = P[7] - P[1], e2z = P[8] - P[2];
    float nx, ny, nz;
    cross3(nx, ny, nz, e1x, e1y, e1z, e2x, e2y, e2z);
    const float r = rsqrt21(nx, ny, nz);
    nx *= r; ny *= r; nz *= r;
    tw[3 * (size_t)i] = make_float4(P[0], P[1], P[2], e1x);
    tw[3 * (size_t)i + 1] = make_float4(e1y, e1z, e2x, e2y);
    tw[3 * (size_t)i + 2] = make_float4(e2z, nx, ny, nz);
    shade[2 * (size_t)i] = make_float4(nx, ny, nz, 0.0f);
    shade[2 * (size_t)i + 1] = make_float4(rad[3 * (size_t)i], rad[3 * (size_t)i + 1], rad[3 * (size_t)i + 2], 0.0f);
}

// init_cam_tri_mem_cuda, TD/Trixel.cu:29-36: d_t = cam - p1, d_q = d_t x e1, d_w = d_q . e2
__global__ void k_cam_tri(const float4* __restrict__ tw, uint32_t ntri, float cx, float cy,
                          float cz, float4* __restrict__ trec) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntri) return;
    const float4 A = tw[3 * (size_t)i], B = tw[3 * (size_t)i + 1], Cq = tw[3 * (size_t)i + 2];
    const float e1x = A.w, e1y = B.x, e1z = B.y, e2x = B.z, e2y = B.w, e2z = Cq.x;
    const float dtx = cx - A.x, dty = cy - A.y, dtz = cz - A.z;
    float qx, qy, qz;
    cross3(qx, qy, qz, dtx, dty, dtz, e1x, e1y, e1z);
    const float dw = dot3(qx, qy, qz, e2x, e2y, e2z);
    trec[4 * (size_t)i] = make_float4(e1x, e1y, e1z, e2x);
    trec[4 * (size_t)i + 1] = make_float4(e2y, e2z, dtx, dty);
    trec[4 * (size_t)i + 2] = make_float4(dtz, qx, qy, qz);
    trec[4 * (size_t)i + 3] = make_float4(dw, 0.0f, 0.0f, 0.0f);
}

// Camera-relative box of a world node, init_cam_voxel_mem_cuda
// (TD/Camera.cu:142-147); obj_center is 0 (TD/Camera.cpp:167-170).
__device__ __forceinline__ void rel_box(const rt_kd_node& nd, float cx, float cy, float cz, float b[6]) {
    const float oc = 0.0f;
    b[0] = nd.x0 - cx + oc; b[1] = nd.x1 - cx + oc;
    b[2] = nd.y0 - cy + oc; b[3] = nd.y1 - cy + oc;
    b[4] = nd.z0 - cz + oc; b[5] = nd.z1 - cz + oc;
}

// Split planes minus the camera on the cut axis, TD/Camera.cu:155-160 (the
// reference's obj_center.x typo on the z term of s2 is kept; it is 0).
__device__ __forceinline__ void rel_split(const rt_kd_node& nd, float cx, float cy, float cz, float& s1,
                                          float& s2, uint32_t& axis) {
    const float ocx = 0.0f, ocy = 0.0f, ocz = 0.0f;
    const int cd = nd.cut_flag;
    const float fx = (cd == 0 || cd == 3) ? 1.0f : 0.0f;
    const float fy = (cd == 1 || cd == 4) ? 1.0f : 0.0f;
    const float fz = (cd == 2 || cd == 5) ? 1.0f : 0.0f;
    s1 = nd.s1 - (((cx + ocx) * fx) + ((cy + ocy) * fy) + ((cz + ocz) * fz));
    s2 = nd.s2 - (((cx + ocx) * fx) + ((cy + ocy) * fy) + ((cz + ocx) * fz));
    axis = fx != 0.0f ? 0u : fy != 0.0f ? 1u : 2u;
}

// The smallest float >= d and the largest float <= d (d a double; NaN stays
// NaN): for a float x, (double)x < d <=> x < ceil_f(d) and (double)x > d <=>
// x > floor_f(d) -- a float between d and its float ceiling would be a
// smaller float >= d.
__device__ __forceinline__ float ceil_f(double d) {
    const float f = (float)d;
    return (double)f < d ? nextafterf(f, INFINITY) : f;
}
__device__ __forceinline__ float floor_f(double d) {
    const float f = (float)d;
    return (double)f > d ? nextafterf(f, -INFINITY) : f;
}

// init_cam_voxel_mem_cuda (TD/Camera.cu:137-162) into the dense interior
// record layout of rt_internal.h (the children's boxes, 64 B).  The split
// word holds the reference's double-promoted split-plane tests as exact float
// thresholds of the camera-relative s2 (TD/Trixel.cu:155-157):
//   (double)mx < (double)s2 + 1e-16  <=>  mx < S_lt = ceil_f(fl64(s2 + 1e-16))
//   (double)mn > (double)s2 - 1e-16  <=>  mn > S_gt = floor_f(fl64(s2 - 1e-16))
// s1 and s2 themselves are the left child's high and the right child's low
// bound on the cut axis (TD/Trixel.h:353-376: the same floats, minus the
// same camera coordinate), read from the boxes where a walk needs them.
// Bit 29 of the right reference marks a node whose s1 is tiny: where
// (float)((double)s1 + 1e-16) differs from s1.
// flags |= kCamTinyS1 when some node's s1 is tiny, kCamUnordered when some
// child box has a low bound not <= its high bound or is not inside its
// parent's box (the kFast walk needs ordered boxes, and its frame proof
// boxes inside the root's: rt_api.cpp fast_proof).
__global__ void k_cam_nodes(const rt_kd_node* __restrict__ nodes, const int32_t* __restrict__ ids,
                            const uint32_t* __restrict__ node_ref, int64_t ninterior, float cx,
                            float cy, float cz, float4* __restrict__ out, int32_t* __restrict__ flags) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ninterior) return;
    const rt_kd_node nd = nodes[ids[k]];
    float s1, s2;
    uint32_t axis;
    rel_split(nd, cx, cy, cz, s1, s2, axis);
    float lb[6], rb[6];
    rel_box(nodes[nd.left], cx, cy, cz, lb);
    rel_box(nodes[nd.right], cx, cy, cz, rb);
    out[4 * k] = make_float4(lb[0], lb[1], lb[2], lb[3]);
    out[4 * k + 1] = make_float4(lb[4], lb[5], rb[0], rb[1]);
    out[4 * k + 2] = make_float4(rb[2], rb[3], rb[4], rb[5]);
    const float s_gt = floor_f((double)s2 - kEps), s_lt = ceil_f((double)s2 + kEps);
    // exactly the records where (float)((double)s1 + 1e-16) is not s1 (bit
    // for bit: zeros, and values within ~2^-29 of zero; NaN)
    const uint32_t tiny = __float_as_uint(pred::add_eps_ref(s1)) == __float_as_uint(s1) ? 0u : kTinyS1Bit;
    float pb[6];
    rel_box(nd, cx, cy, cz, pb);
    bool ordered = true;
    for (int a = 0; a < 3; a++)
        ordered = ordered && lb[2 * a] <= lb[2 * a + 1] && rb[2 * a] <= rb[2 * a + 1] && lb[2 * a] >= pb[2 * a] &&
                  rb[2 * a] >= pb[2 * a] && lb[2 * a + 1] <= pb[2 * a + 1] && rb[2 * a + 1] <= pb[2 * a + 1];
    const int32_t f = (tiny ? kCamTinyS1 : 0) | (ordered ? 0 : kCamUnordered);
    if (f) atomicOr(flags, f);
    out[4 * k + 3] = make_float4(s_gt, s_lt, __uint_as_float(node_ref[nd.left] | (axis << kAxisShift)),
                                 __uint_as_float(node_ref[nd.right] | tiny));
}

// Rank 0's frame assembly after the gather: [rank][slot][8 rows][w] -> frame.
// Every frame row is one contiguous row of the gathered buffer, so a block
// copies one row (blockIdx.y) in 16-byte pieces when the rows are 16-byte
// aligned (w % 4 == 0 and 16-byte aligned buffers: vec), else word by word.
__global__ void k_unpack(int32_t w, int32_t h, int32_t nranks, int32_t slots, int32_t vec,
                         const uint32_t* __restrict__ g, uint32_t* __restrict__ frame) {
    const int32_t y = blockIdx.y;
    const int32_t band = y / kTileH, r = y - band * kTileH;
    const int32_t rank = band % nranks, slot = band / nranks;
    const uint32_t* src = g + (((int64_t)rank * slots + slot) * kTileH + r) * w;
    uint32_t* dst = frame + (int64_t)y * w;
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (vec) {
        if (i < (w >> 2)) reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    } else {
        for (int32_t k = i; k < w; k += gridDim.x * blockDim.x) dst[k] = src[k];
    }
}

// The rectangle gather (rt_frame_rect): outside columns [x0, x1) of bands
// [b0, b1) every pixel is provably background, so a rank sends only its
// slots' rows inside the rectangle.  Pack: row (s - s0)*8 + r of the
// compact buffer <- columns [x0, x1) of packed row s*8 + r.
__global__ void k_pack_rect(int32_t w, int32_t x0, int32_t cw, int32_t s0, const uint32_t* __restrict__ local,
                            uint32_t* __restrict__ out) {
    const int32_t row = blockIdx.y;
    const int32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= cw) return;
    const int32_t s = s0 + row / kTileH, r = row - (row / kTileH) * kTileH;
    out[(int64_t)row * cw + x] = local[((int64_t)s * kTileH + r) * w + x0 + x];
}

// Rank 0: frame rows y0 + blockIdx.y * rpb ... (rpb of them, within rows)
// from rank 0's own packed buffer, a peer's compact block (peers 1..N-1 back
// to back), or the background.
// Each thread writes `vec` (4 or 1) consecutive pixels of the row from
// column xa; rows outside the rectangle are pure background stores.  The
// whole frame: y0 = xa = 0; the rectangle alone (its background already in
// the frame): its rows, from column x0 rounded down to a multiple of vec.
// local0 = null: rank 0's rows are in the frame already (RT_FLAG_FRAME_OUT).
__global__ void k_unpack_rect(int32_t w, int32_t nranks, int32_t x0, int32_t x1, int32_t b0, int32_t b1, int32_t vec,
                              int32_t y0, int32_t xa, int32_t rows, int32_t rpb, const uint32_t* __restrict__ local0,
                              const uint32_t* __restrict__ peers, uint32_t* __restrict__ frame) {
    const int32_t xs = xa + (blockIdx.x * blockDim.x + threadIdx.x) * vec;
    if (xs >= w) return;
    const int32_t ye = y0 + min(rows, (int32_t)(blockIdx.y + 1) * rpb);
    for (int32_t y = y0 + (int32_t)blockIdx.y * rpb; y < ye; y++) {
        const int32_t band = y / kTileH, r = y - band * kTileH;
        const int32_t rank = band % nranks, slot = band / nranks;
        if (rank == 0 && !local0) continue;  // rank 0 rendered these rows into the frame
        uint32_t v0 = kBackground, v1 = kBackground, v2 = kBackground, v3 = kBackground;
        if (band >= b0 && band < b1 && xs + vec > x0 && xs < x1) {
            const uint32_t* src;
            int32_t sx;  // source index of column x: src[x - sx]
            if (rank == 0) {
                src = local0 + ((int64_t)slot * kTileH + r) * w;
                sx = 0;
            } else {
                const int32_t cw = x1 - x0;
                int64_t off = 0;
                int32_t s0, s1;
                for (int32_t q = 1; q < rank; q++) {
                    rect_slots(b0, b1, nranks, q, s0, s1);
                    off += (int64_t)(s1 - s0) * kTileH * cw;
                }
                rect_slots(b0, b1, nranks, rank, s0, s1);
                src = peers + off + ((int64_t)(slot - s0) * kTileH + r) * cw;
                sx = x0;
            }
            // straight-line per pixel (an indexed array would live in scratch)
            if (xs >= x0 && xs < x1) v0 = src[xs - sx];
            if (vec == 4) {
                if (xs + 1 >= x0 && xs + 1 < x1) v1 = src[xs + 1 - sx];
                if (xs + 2 >= x0 && xs + 2 < x1) v2 = src[xs + 2 - sx];
                if (xs + 3 >= x0 && xs + 3 < x1) v3 = src[xs + 3 - sx];
            }
        }
        uint32_t* dst = frame + (int64_t)y * w + xs;
        if (vec == 4) {
            *reinterpret_cast<uint4*>(dst) = make_uint4(v0, v1, v2, v3);
        } else {
            dst[0] = v0;
        }
    }
}

template <class K>
int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(RT_ERR_HIP, "%s launch failed: %s", what, hipGetErrorString(e));
    return RT_OK;
}

using TraceFn = void (*)(TraceParams);

template <bool T, bool H, bool C, int S>
TraceFn kd3_kernel(int rays, bool coarse) {
    if (coarse) {
        if (rays == 8) return k_coarse_kd3<8, T, H, C, S>;
        if (rays == 16) return k_coarse_kd3<16, T, H, C, S>;
        return k_coarse_kd3<32, T, H, C, S>;
    }
    if (rays == 8) return k_trace_kd3<8, T, H, C, S>;
    if (rays == 16) return k_trace_kd3<16, T, H, C, S>;
    return k_trace_kd3<32, T, H, C, S>;
}

// shadow: -1 none, else the any-hit push order (0..3), + 4 for counting
// walks that stop at occluders like a timed frame's (bench.py's roofline).
// Other counting walks are not cut short, so the order does not change their
// work: one instance serves them.
template <bool T, bool H, bool C>
TraceFn kd_kernel(int version, int rays, int shadow, bool coarse) {
    if (version == 2) return k_trace_kd2<T, H, C>;
    if (shadow < 0) return kd3_kernel<T, H, C, 0>(rays, coarse);
    if constexpr (C) {
        switch (shadow) {
        case 4: return kd3_kernel<T, H, C, 5>(rays, coarse);
        case 5: return kd3_kernel<T, H, C, 6>(rays, coarse);
        case 6: return kd3_kernel<T, H, C, 7>(rays, coarse);
        case 7: return kd3_kernel<T, H, C, 8>(rays, coarse);
        default: return kd3_kernel<T, H, C, 1>(rays, coarse);
        }
    } else {
        shadow &= 3;
        switch (shadow) {
        case 0: return kd3_kernel<T, H, C, 1>(rays, coarse);
        case 1: return kd3_kernel<T, H, C, 2>(rays, coarse);
        case 2: return kd3_kernel<T, H, C, 3>(rays, coarse);
        default: return kd3_kernel<T, H, C, 4>(rays, coarse);
        }
    }
}

}  // namespace
}  // namespace rt
