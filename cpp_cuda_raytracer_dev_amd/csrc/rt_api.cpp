// rt_api.cpp -- the C ABI (include/rt_mi355x.h) over the HIP runtime.
//
// Handles own every device buffer they allocate and free it in rt_*_destroy
// (the reference never frees: TD/Camera.cpp:143-210, TD/Trixel.h:90-124).
// Every launch is stream-ordered and checked with hipGetLastError; nothing on
// the render path synchronises or allocates, so a caller may capture
// rt_render_into in a hipGraph.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "rt_internal.h"

using namespace rt;

struct rt_scene {
    int device = 0;
    uint32_t ntri = 0;
    float4* d_tri_world = nullptr;   // (p1, e1, e2, n) per triangle
    float4* d_shade = nullptr;       // (n, rad) per triangle
    rt_kd_node* d_nodes = nullptr;   // world-space tree as uploaded
    int32_t* d_interior_ids = nullptr;
    uint32_t* d_node_ref = nullptr;
    int64_t nnode = 0, ninterior = 0;
    uint32_t root_ref = 0;
    int32_t height = 0;
    uint64_t tree_version = 0;
    rt_kd_node root{};               // host copy of node 0 (root box)
};

struct rt_camera {
    int device = 0;
    int32_t w = 0, h = 0;
    float pos[3] = {0, 0, 0};
    rt_camera_basis_t basis{};
    uint32_t* d_argb = nullptr;
    int64_t* d_hit = nullptr;
    unsigned long long* d_counters = nullptr;
    int32_t* d_err = nullptr;
    rt_scene* obj = nullptr;
    uint64_t prepared_version = 0;
    float4* d_trec = nullptr;        // camera-relative triangle records
    float4* d_inode = nullptr;       // camera-relative interior nodes
    uint32_t trec_cap = 0;
    int64_t inode_cap = 0;           // in float4
    int prepared_layout = 0;         // interior record layout of d_inode (1 or 2)
    int kernel_version = 3;          // kOptKernel (3 falls back to 2 on trees taller than 21)
    int tile_order = 2;              // kOptTileOrder
    int debug = 0;                   // kOptDebug (diagnostics)
    int pool_cap = kPoolCapMax;      // kOptPoolCap
    unsigned long long* d_dbg = nullptr;
    int64_t dbg_cap = 0;             // in u64
    int32_t* d_order = nullptr;      // centre-out tile permutation
    int64_t order_cap = 0;
    int64_t order_key[6] = {-1, -1, -1, -1, -1, -1};
    int rays = 16;                   // kOptRays: pixels per wave of kernel 3
    int items = 2;                   // kOptItems: items per lane per pool iteration
};

namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return RT_OK;
    return fail(e == hipErrorOutOfMemory ? RT_ERR_NOMEM : RT_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

template <class T>
int dev_alloc(T** p, size_t count, const char* what) {
    *p = nullptr;
    if (count == 0) count = 1;
    return hip_check(hipMalloc((void**)p, sizeof(T) * count), what);
}

template <class T>
void dev_free(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

// The KD kernel a render runs: the wave-cooperative kernel (3) encodes DFS
// path codes in 21 bits, so taller trees use the per-lane DFS kernel (2).
int effective_kernel(const rt_camera* c) {
    if (c->kernel_version == 3 && c->obj && c->obj->height > 21) return 2;
    return c->kernel_version;
}

int record_layout(int kernel) { return kernel == 1 ? 1 : 2; }

int prepare_camera_object(rt_camera* c) {
    rt_scene* s = c->obj;
    if (!s) return fail(RT_ERR_STATE, "camera has no object (rt_camera_add_object)");
    const int layout = record_layout(effective_kernel(c));
    if (c->prepared_version == s->tree_version + 1 && c->prepared_layout == layout) return RT_OK;
    int rc;
    if (c->trec_cap < s->ntri) {
        dev_free(c->d_trec);
        if ((rc = dev_alloc(&c->d_trec, (size_t)s->ntri * 4, "hipMalloc(trec)"))) return rc;
        c->trec_cap = s->ntri;
    }
    // init_camera_trixel_device_memory (TD/Trixel.cu:244-264)
    if ((rc = launch_cam_tri(s->d_tri_world, s->ntri, c->pos, c->d_trec, nullptr))) return rc;
    if (s->d_nodes) {
        const int64_t need = std::max<int64_t>(s->ninterior, 1) * (layout == 1 ? 3 : 4);
        if (c->inode_cap < need) {
            dev_free(c->d_inode);
            if ((rc = dev_alloc(&c->d_inode, (size_t)need, "hipMalloc(inode)"))) return rc;
            c->inode_cap = need;
        }
        // init_camera_voxel_device_memory (TD/Camera.cu:163-187)
        if ((rc = launch_cam_nodes(s->d_nodes, s->d_interior_ids, s->d_node_ref, s->ninterior, c->pos,
                                   c->d_inode, layout, nullptr)))
            return rc;
    }
    if ((rc = hip_check(hipDeviceSynchronize(), "camera object prep"))) return rc;
    c->prepared_version = s->tree_version + 1;
    c->prepared_layout = layout;
    return RT_OK;
}

// Centre-out permutation of the launch's tiles: blocks are dispatched in
// index order, so the expensive tiles (the object sits mid-frame) start
// first and the cheap background tiles fill in behind them.
int ensure_order(rt_camera* c, const TraceParams& p) {
    const int64_t key[6] = {p.tile_w, p.tile_h, p.tiles_x, p.block_rows, p.nranks, p.rank};
    if (std::equal(key, key + 6, c->order_key)) return RT_OK;
    const int64_t n = (int64_t)p.tiles_x * p.block_rows;
    const int64_t per_band = kTileH / p.tile_h;
    std::vector<int32_t> order((size_t)n);
    std::vector<double> dist2((size_t)n);
    const double cx = 0.5 * c->w, cy = 0.5 * c->h;
    for (int64_t t = 0; t < n; t++) {
        const int64_t row = t / p.tiles_x, tx = t % p.tiles_x;
        const int64_t slot = row / per_band, yin = (row % per_band) * p.tile_h;
        const double x = (tx + 0.5) * p.tile_w;
        const double y = (double)((p.rank + slot * (int64_t)p.nranks) * kTileH + yin) + 0.5 * p.tile_h;
        dist2[(size_t)t] = (x - cx) * (x - cx) + (y - cy) * (y - cy);
        order[(size_t)t] = (int32_t)t;
    }
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return dist2[(size_t)a] < dist2[(size_t)b]; });
    int rc;
    if (c->order_cap < n) {
        dev_free(c->d_order);
        if ((rc = dev_alloc(&c->d_order, (size_t)n, "hipMalloc(order)"))) return rc;
        c->order_cap = n;
    }
    if ((rc = hip_check(hipMemcpy(c->d_order, order.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice), "H2D order")))
        return rc;
    std::copy(key, key + 6, c->order_key);
    return RT_OK;
}

int fill_params(rt_camera* c, const float* xform, const rt_tile* tile, uint32_t* argb, int64_t* hit,
                uint32_t mode, TraceParams& p) {
    static const float ident[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const rt_scene* s = c->obj;
    p.inode = c->d_inode;
    p.trec = c->d_trec;
    p.shade = s->d_shade;
    p.argb = argb;
    p.hit = hit;
    p.counters = c->d_counters;
    p.err = c->d_err;
    for (int k = 0; k < 3; k++) {
        p.n_mod[k] = c->basis.n_mod[k];
        p.u_mod[k] = c->basis.u_mod[k];
        p.v_mod[k] = c->basis.v_mod[k];
    }
    memcpy(p.xf, xform ? xform : ident, sizeof p.xf);
    p.w = c->w;
    p.h = c->h;
    p.nranks = tile ? tile->nranks : 1;
    p.rank = tile ? tile->rank : 0;
    const int32_t nbands = (c->h + kTileH - 1) / kTileH;
    const int kernel = mode == RT_MODE_KD ? effective_kernel(c) : 0;
    p.rays = kernel == 3 ? c->rays : 64;
    if (kernel == 0 || kernel == 1) {        // flat / v1: 32x8 tiles, four 8x8 waves
        p.tile_w = kTileWFlat; p.tile_h = kTileH;
    } else if (p.rays == 64) {               // v2 / v3: 16x8 tiles, two 8x8 waves
        p.tile_w = kTileWKd; p.tile_h = kTileH;
    } else {                                 // v3, two stacked 8 x (rays/8) waves
        p.tile_w = 8; p.tile_h = 2 * (p.rays / 8);
    }
    p.tiles_x = (c->w + p.tile_w - 1) / p.tile_w;
    p.block_rows = ((nbands + p.nranks - 1) / p.nranks) * (kTileH / p.tile_h);
    p.root_ref = s->root_ref;
    p.ntri = s->ntri;
    p.max_depth = kMaxDepth;
    p.tile_order = c->tile_order;
    p.order = nullptr;
    p.debug = c->debug;
    p.pool_cap = c->pool_cap;
    p.items = c->items;
    p.dbg = nullptr;
    if (c->debug & 2) {
        const int64_t need = (int64_t)p.tiles_x * p.block_rows * 4 * 3;  // <= 4 waves per block
        if (c->dbg_cap < need) {
            dev_free(c->d_dbg);
            int rc = dev_alloc(&c->d_dbg, (size_t)need, "hipMalloc(dbg)");
            if (rc) return rc;
            c->dbg_cap = need;
        }
        p.dbg = c->d_dbg;
        int rc = hip_check(hipMemset(c->d_dbg, 0, sizeof(uint64_t) * (size_t)need), "memset dbg");
        if (rc) return rc;
    }
    camera_relative_box(s->root, c->pos, p.root_box);
    if (c->tile_order == 2) {
        int rc = ensure_order(c, p);
        if (rc) return rc;
        p.order = c->d_order;
    }
    return RT_OK;
}

int check_tile(const rt_tile* tile) {
    if (tile && (tile->nranks < 1 || tile->rank < 0 || tile->rank >= tile->nranks))
        return fail(RT_ERR_INVALID, "rt_tile: rank %d of %d", tile->rank, tile->nranks);
    return RT_OK;
}

}  // namespace

extern "C" int rt_device_count(int* count) {
    if (!count) return fail(RT_ERR_INVALID, "rt_device_count: null");
    return hip_check(hipGetDeviceCount(count), "hipGetDeviceCount");
}

extern "C" int rt_scene_create(int device, const float* points9, const float* rad3, uint32_t ntri,
                               rt_scene** out) {
    if (!out || (ntri && (!points9 || !rad3))) return fail(RT_ERR_INVALID, "rt_scene_create: null argument");
    if (ntri > kRefMask) return fail(RT_ERR_INVALID, "rt_scene_create: more than 2^29 triangles");
    *out = nullptr;
    DeviceGuard g(device);
    if (!g.ok) return fail(RT_ERR_HIP, "rt_scene_create: hipSetDevice(%d) failed", device);
    rt_scene* s = new rt_scene();
    s->device = device;
    s->ntri = ntri;
    float *d_pts = nullptr, *d_rad = nullptr;
    int rc;
    if ((rc = dev_alloc(&s->d_tri_world, (size_t)ntri * 3, "hipMalloc(tri_world)")) ||
        (rc = dev_alloc(&s->d_shade, (size_t)ntri * 2, "hipMalloc(shade)")) ||
        (rc = dev_alloc(&d_pts, (size_t)ntri * 9, "hipMalloc(points)")) ||
        (rc = dev_alloc(&d_rad, (size_t)ntri * 3, "hipMalloc(rad)")) ||
        (rc = hip_check(hipMemcpy(d_pts, points9, sizeof(float) * 9 * ntri, hipMemcpyHostToDevice), "H2D points")) ||
        (rc = hip_check(hipMemcpy(d_rad, rad3, sizeof(float) * 3 * ntri, hipMemcpyHostToDevice), "H2D rad")) ||
        (rc = launch_tri_world(d_pts, d_rad, ntri, s->d_tri_world, s->d_shade, nullptr)) ||
        (rc = hip_check(hipDeviceSynchronize(), "init_tri_mem"))) {
        dev_free(d_pts);
        dev_free(d_rad);
        rt_scene_destroy(s);
        return rc;
    }
    dev_free(d_pts);
    dev_free(d_rad);
    *out = s;
    return RT_OK;
}

extern "C" int rt_scene_set_kd(rt_scene* s, const rt_kd_node* nodes, uint64_t nnode) {
    if (!s || !nodes) return fail(RT_ERR_INVALID, "rt_scene_set_kd: null argument");
    const int64_t n = (int64_t)nnode;
    if (s->ntri == 0 || n != 2 * (int64_t)s->ntri - 1)
        return fail(RT_ERR_INVALID, "rt_scene_set_kd: %lld nodes for %u triangles", (long long)n, s->ntri);
    // Validate: BFS order with right = left + 1 (so every DFS terminates),
    // leaves cover every triangle exactly once, bounded height.
    std::vector<uint32_t> ref((size_t)n);
    std::vector<int32_t> ids;
    std::vector<uint8_t> seen(s->ntri, 0);
    std::vector<int32_t> depth((size_t)n, 0);
    int64_t ninterior = 0;
    int32_t height = 0;
    for (int64_t i = 0; i < n; i++) {
        const rt_kd_node& nd = nodes[i];
        if (nd.is_leaf) {
            if (nd.tri_index < 0 || nd.tri_index >= (int64_t)s->ntri || seen[(size_t)nd.tri_index])
                return fail(RT_ERR_INVALID, "rt_scene_set_kd: leaf %lld has bad/duplicate triangle", (long long)i);
            seen[(size_t)nd.tri_index] = 1;
            ref[(size_t)i] = kLeafBit | (uint32_t)nd.tri_index;
        } else {
            if (nd.left <= i || nd.right != nd.left + 1 || nd.right >= n)
                return fail(RT_ERR_INVALID, "rt_scene_set_kd: node %lld children %lld/%lld not BFS", (long long)i,
                            (long long)nd.left, (long long)nd.right);
            if (nd.cut_flag < 0 || nd.cut_flag > 5)
                return fail(RT_ERR_INVALID, "rt_scene_set_kd: node %lld cut_flag %d", (long long)i, nd.cut_flag);
            depth[(size_t)nd.left] = depth[(size_t)i] + 1;
            depth[(size_t)nd.right] = depth[(size_t)i] + 1;
            height = std::max(height, depth[(size_t)i] + 1);
            ref[(size_t)i] = (uint32_t)ninterior++;
            ids.push_back((int32_t)i);
        }
    }
    if (height > kMaxDepth)
        return fail(RT_ERR_INVALID, "rt_scene_set_kd: tree height %d exceeds the %d-entry LDS stack", height, kMaxDepth);
    DeviceGuard g(s->device);
    dev_free(s->d_nodes);
    dev_free(s->d_interior_ids);
    dev_free(s->d_node_ref);
    int rc;
    if ((rc = dev_alloc(&s->d_nodes, (size_t)n, "hipMalloc(nodes)")) ||
        (rc = dev_alloc(&s->d_interior_ids, ids.size(), "hipMalloc(ids)")) ||
        (rc = dev_alloc(&s->d_node_ref, (size_t)n, "hipMalloc(node_ref)")) ||
        (rc = hip_check(hipMemcpy(s->d_nodes, nodes, sizeof(rt_kd_node) * (size_t)n, hipMemcpyHostToDevice), "H2D nodes")) ||
        (rc = hip_check(hipMemcpy(s->d_node_ref, ref.data(), sizeof(uint32_t) * (size_t)n, hipMemcpyHostToDevice), "H2D refs")) ||
        (!ids.empty() && (rc = hip_check(hipMemcpy(s->d_interior_ids, ids.data(), sizeof(int32_t) * ids.size(),
                                                   hipMemcpyHostToDevice), "H2D ids")))) {
        dev_free(s->d_nodes);
        return rc;
    }
    s->nnode = n;
    s->root = nodes[0];
    s->ninterior = ninterior;
    s->root_ref = ref[0];
    s->height = height;
    s->tree_version++;
    return RT_OK;
}

extern "C" int rt_camera_create(int device, int32_t w, int32_t h, float f_w, float f_h, float focal,
                                const float pos[3], const float look_at[3], const float up[3],
                                rt_camera** out) {
    if (!out) return fail(RT_ERR_INVALID, "rt_camera_create: null out");
    *out = nullptr;
    if (w <= 0 || h <= 0 || (int64_t)w * h > (int64_t)1 << 31)
        return fail(RT_ERR_INVALID, "rt_camera_create: bad resolution %dx%d", w, h);
    rt_camera_basis_t basis;
    int rc = rt_camera_basis(w, h, f_w, f_h, focal, pos, look_at, up, &basis);
    if (rc) return rc;
    DeviceGuard g(device);
    if (!g.ok) return fail(RT_ERR_HIP, "rt_camera_create: hipSetDevice(%d) failed", device);
    rt_camera* c = new rt_camera();
    c->device = device;
    c->w = w;
    c->h = h;
    for (int k = 0; k < 3; k++) c->pos[k] = pos[k];
    c->basis = basis;
    const size_t npix = (size_t)w * h;
    if ((rc = dev_alloc(&c->d_argb, npix, "hipMalloc(argb)")) ||
        (rc = dev_alloc(&c->d_hit, npix, "hipMalloc(hit)")) ||
        (rc = dev_alloc(&c->d_counters, 5, "hipMalloc(counters)")) ||
        (rc = dev_alloc(&c->d_err, 1, "hipMalloc(err)")) ||
        // init_cam_mem_cuda (TD/Camera.cu:97-110): frame zeroed, rmi = -1
        (rc = hip_check(hipMemset(c->d_argb, 0, npix * sizeof(uint32_t)), "memset argb")) ||
        (rc = hip_check(hipMemset(c->d_hit, 0xFF, npix * sizeof(int64_t)), "memset hit")) ||
        (rc = hip_check(hipMemset(c->d_counters, 0, 5 * sizeof(unsigned long long)), "memset counters")) ||
        (rc = hip_check(hipMemset(c->d_err, 0, sizeof(int32_t)), "memset err"))) {
        rt_camera_destroy(c);
        return rc;
    }
    *out = c;
    return RT_OK;
}

extern "C" int rt_camera_add_object(rt_camera* c, rt_scene* s) {
    if (!c || !s) return fail(RT_ERR_INVALID, "rt_camera_add_object: null argument");
    if (c->device != s->device) return fail(RT_ERR_INVALID, "rt_camera_add_object: camera and scene on different devices");
    DeviceGuard g(c->device);
    c->obj = s;
    c->prepared_version = 0;
    return prepare_camera_object(c);
}

static int render_common(rt_camera* c, const float* xform, uint32_t mode, uint32_t flags, const rt_tile* tile,
                         uint32_t* argb, int64_t* hit, void* stream) {
    if (!c) return fail(RT_ERR_INVALID, "rt_render: null camera");
    if (mode != RT_MODE_KD && mode != RT_MODE_FLAT) return fail(RT_ERR_INVALID, "rt_render: mode %u", mode);
    int rc = check_tile(tile);
    if (rc) return rc;
    if (!argb || ((flags & RT_FLAG_WRITE_HIT) && !hit)) return fail(RT_ERR_INVALID, "rt_render: null output buffer");
    DeviceGuard g(c->device);
    if ((rc = prepare_camera_object(c))) return rc;
    if (mode == RT_MODE_KD && !c->obj->d_nodes)
        return fail(RT_ERR_STATE, "rt_render: KD mode needs rt_scene_set_kd (Trixel::create_kd) first");
    if (c->obj->ntri == 0) return fail(RT_ERR_STATE, "rt_render: empty scene");
    if (flags & ~(RT_FLAG_WRITE_HIT | RT_FLAG_COUNT | RT_FLAG_SHADOW))
        return fail(RT_ERR_INVALID, "rt_render: unknown flags 0x%x", flags);
    if (flags & RT_FLAG_SHADOW) {
        if (mode != RT_MODE_KD) return fail(RT_ERR_INVALID, "rt_render: RT_FLAG_SHADOW needs RT_MODE_KD");
        if (effective_kernel(c) != 3)
            return fail(RT_ERR_STATE, "rt_render: shadow rays run in the wave-cooperative kernel (3); kernel %d%s",
                        effective_kernel(c), c->obj->height > 21 ? " (tree height > 21)" : "");
    }
    TraceParams p;
    if ((rc = fill_params(c, xform, tile, argb, hit, mode, p))) return rc;
    return launch_trace(p, mode, flags, effective_kernel(c), stream);
}

extern "C" int rt_render(rt_camera* c, const float* xform, uint32_t mode, uint32_t flags, const rt_tile* tile,
                         void* stream) {
    if (!c) return fail(RT_ERR_INVALID, "rt_render: null camera");
    if (tile && tile->nranks != 1)
        return fail(RT_ERR_INVALID, "rt_render: the camera's own buffer holds a full frame; use rt_render_into for tiles");
    return render_common(c, xform, mode, flags, tile, c->d_argb, c->d_hit, stream);
}

extern "C" int rt_render_into(rt_camera* c, const float* xform, uint32_t mode, uint32_t flags, const rt_tile* tile,
                              uint32_t* d_argb, int64_t* d_hit, void* stream) {
    return render_common(c, xform, mode, flags, tile, d_argb, d_hit, stream);
}

extern "C" int64_t rt_tile_packed_pixels(int32_t w, int32_t h, int32_t nranks) {
    if (w <= 0 || h <= 0 || nranks < 1) return -1;
    const int64_t nbands = (h + kTileH - 1) / kTileH;
    const int64_t slots = (nbands + nranks - 1) / nranks;
    return slots * kTileH * (int64_t)w;
}

extern "C" int rt_unpack_bands(int device, int32_t w, int32_t h, int32_t nranks, const uint32_t* d_gathered,
                               uint32_t* d_frame, void* stream) {
    if (!d_gathered || !d_frame || w <= 0 || h <= 0 || nranks < 1) return fail(RT_ERR_INVALID, "rt_unpack_bands: bad argument");
    DeviceGuard g(device);
    return launch_unpack(w, h, nranks, d_gathered, d_frame, stream);
}

extern "C" int rt_read_frame(rt_camera* c, uint32_t* argb, int64_t* hit) {
    if (!c || !argb) return fail(RT_ERR_INVALID, "rt_read_frame: null argument");
    DeviceGuard g(c->device);
    int rc;
    if ((rc = hip_check(hipDeviceSynchronize(), "rt_read_frame sync"))) return rc;
    int32_t err = 0;
    if ((rc = hip_check(hipMemcpy(&err, c->d_err, sizeof err, hipMemcpyDeviceToHost), "D2H err"))) return rc;
    const size_t npix = (size_t)c->w * c->h;
    if ((rc = hip_check(hipMemcpy(argb, c->d_argb, npix * sizeof(uint32_t), hipMemcpyDeviceToHost), "D2H argb")))
        return rc;
    if (hit && (rc = hip_check(hipMemcpy(hit, c->d_hit, npix * sizeof(int64_t), hipMemcpyDeviceToHost), "D2H hit")))
        return rc;
    if (err) return fail(RT_ERR_OVERFLOW, "traversal stack overflow reported by the device");
    return RT_OK;
}

extern "C" int rt_camera_counters(rt_camera* c, uint64_t out[5], int reset) {
    if (!c || !out) return fail(RT_ERR_INVALID, "rt_camera_counters: null argument");
    DeviceGuard g(c->device);
    int rc;
    if ((rc = hip_check(hipDeviceSynchronize(), "counters sync"))) return rc;
    unsigned long long tmp[5];
    if ((rc = hip_check(hipMemcpy(tmp, c->d_counters, sizeof tmp, hipMemcpyDeviceToHost), "D2H counters"))) return rc;
    for (int k = 0; k < 5; k++) out[k] = tmp[k];
    if (reset && (rc = hip_check(hipMemset(c->d_counters, 0, sizeof tmp), "reset counters"))) return rc;
    int32_t err = 0;
    if ((rc = hip_check(hipMemcpy(&err, c->d_err, sizeof err, hipMemcpyDeviceToHost), "D2H err"))) return rc;
    if (err) return fail(RT_ERR_OVERFLOW, "traversal stack overflow reported by the device");
    return RT_OK;
}

extern "C" int rt_camera_info(const rt_camera* c, int32_t* w, int32_t* h, int32_t* max_depth) {
    if (!c) return fail(RT_ERR_INVALID, "rt_camera_info: null camera");
    if (w) *w = c->w;
    if (h) *h = c->h;
    if (max_depth) *max_depth = c->obj ? c->obj->height : 0;
    return RT_OK;
}

extern "C" void rt_scene_destroy(rt_scene* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    dev_free(s->d_tri_world);
    dev_free(s->d_shade);
    dev_free(s->d_nodes);
    dev_free(s->d_interior_ids);
    dev_free(s->d_node_ref);
    delete s;
}

extern "C" void rt_camera_destroy(rt_camera* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    dev_free(c->d_argb);
    dev_free(c->d_hit);
    dev_free(c->d_counters);
    dev_free(c->d_err);
    dev_free(c->d_trec);
    dev_free(c->d_inode);
    dev_free(c->d_order);
    dev_free(c->d_dbg);
    delete c;
}

extern "C" int rt_camera_set_option(rt_camera* c, int32_t key, int32_t value) {
    if (!c) return fail(RT_ERR_INVALID, "rt_camera_set_option: null camera");
    switch (key) {
    case kOptKernel:
        if (value < 1 || value > 3) return fail(RT_ERR_INVALID, "kernel version %d", value);
        c->kernel_version = value;
        return RT_OK;
    case kOptRays:
        if (value != 16 && value != 32 && value != 64) return fail(RT_ERR_INVALID, "rays per wave %d (16, 32, 64)", value);
        c->rays = value;
        return RT_OK;
    case kOptItems:
        if (value != 1 && value != 2) return fail(RT_ERR_INVALID, "items per lane %d (1, 2)", value);
        c->items = value;
        return RT_OK;
    case kOptPoolCap:
        // the 64 root items plus a DFS run of height <= 21 must fit
        if (value < 64 + 22 || value > kPoolCapMax)
            return fail(RT_ERR_INVALID, "pool cap %d (86..%d)", value, kPoolCapMax);
        c->pool_cap = value;
        return RT_OK;
    case kOptDebug:
        c->debug = value;
        return RT_OK;
    case kOptTileOrder:
        if (value < 0 || value > 2) return fail(RT_ERR_INVALID, "tile order %d", value);
        c->tile_order = value;
        return RT_OK;
    default:
        return fail(RT_ERR_INVALID, "rt_camera_set_option: unknown key %d", key);
    }
}

namespace rt {
void camera_relative_box(const rt_kd_node& nd, const float pos[3], float b[6]) {
    // init_cam_voxel_mem_cuda, TD/Camera.cu:142-147 (obj_center = 0); the
    // same IEEE operations as the device-side rel_box
    const float oc = 0.0f;
    b[0] = nd.x0 - pos[0] + oc; b[1] = nd.x1 - pos[0] + oc;
    b[2] = nd.y0 - pos[1] + oc; b[3] = nd.y1 - pos[1] + oc;
    b[4] = nd.z0 - pos[2] + oc; b[5] = nd.z1 - pos[2] + oc;
}
}  // namespace rt

extern "C" int64_t rt_camera_debug_read(rt_camera* c, uint64_t* out, int64_t n) {
    if (!c || !out || !c->d_dbg) return fail(RT_ERR_STATE, "rt_camera_debug_read: no diagnostic buffer");
    DeviceGuard g(c->device);
    const int64_t m = std::min(n, c->dbg_cap);
    if (hip_check(hipDeviceSynchronize(), "debug sync") ||
        hip_check(hipMemcpy(out, c->d_dbg, sizeof(uint64_t) * (size_t)m, hipMemcpyDeviceToHost), "D2H dbg"))
        return RT_ERR_HIP;
    return m;
}
