// kd_build_gpu.hip -- the reference's KD build on the GPU, producing the
// identical node array.
//
// The reference builds on the host: Trixel::set_sorted_voxels
// (TD/Trixel.h:386-473) merge-sorts the leaf boxes six times (TD/sort.h:11-60,
// the right run first on ties), and Trixel::create_kd (TD/Trixel.h:135-385)
// splits BFS-level by level at the position median, stably partitioning the
// other five lists (:214-327).  rt_kd_build (scene_host.cpp) restates that on
// host threads; this is the same algorithm laid out for the GPU:
//
//  * the tree's shape (every node's position range, children, level) depends
//    on n alone -- a range of s elements splits into ceil(s/2) and floor(s/2)
//    -- so the host lays it out once and no level needs a host round trip;
//  * the six sorts are stable LSD radix sorts (rocPRIM) of the keys fed in
//    descending position order, which is merge_sort's tie order (key
//    ascending, position descending); -0.0 is sorted as +0.0, since the
//    reference compares with `<`;
//  * a level's stable partitions are one exclusive scan over all six lists of
//    the "goes left" flags (ranges are disjoint, so a node's rank of an
//    element is a difference of the global scan) and one scatter;
//  * every float operation (the spans of the cut choice) is the host's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <vector>

#include "rt_internal.h"

namespace rt {
namespace {

constexpr int kBlk = 256;

// Lists in cut-flag order (TD/Trixel.h:172-193): 0 x1, 1 y1, 2 z1, 3 x0, 4 y0, 5 z0.
__device__ __forceinline__ float list_key_d(const rt_leaf_aabb& a, int k) {
    switch (k) {
    case 0: return a.x1;
    case 1: return a.y1;
    case 2: return a.z1;
    case 3: return a.x0;
    case 4: return a.y0;
    default: return a.z0;
    }
}

// Order-preserving unsigned image of a non-NaN float, -0.0 as +0.0.
__device__ __forceinline__ uint32_t sortable(float f) {
    uint32_t u = __float_as_uint(f);
    if (f == 0.0f) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Sort input of list k: positions in descending order with their keys.
__global__ void k_sort_input(const rt_leaf_aabb* __restrict__ lf, uint32_t n, int k, uint32_t* __restrict__ keys,
                             uint32_t* __restrict__ vals) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t pos = n - 1 - j;
    keys[j] = sortable(list_key_d(lf[pos], k));
    vals[j] = pos;
}

struct Lists {
    const uint32_t* L;  // 6 lists of n positions, back to back
    uint32_t n;
    __device__ __forceinline__ uint32_t at(int k, int64_t p) const { return L[(size_t)k * n + (size_t)p]; }
};

__device__ __forceinline__ float key_at(const rt_leaf_aabb* lf, const Lists& S, int k, int64_t p) {
    return list_key_d(lf[S.at(k, p)], k);
}

// The root (TD/Trixel.h:135-160): its box from the sorted lists.
__global__ void k_root(const rt_leaf_aabb* __restrict__ lf, Lists S, rt_kd_node* __restrict__ nodes) {
    const int64_t n = S.n;
    rt_kd_node& r = nodes[0];
    r.parent = 0;
    r.cut_flag = 5;
    r.tri_index = -1;
    r.is_leaf = 0;
    r.left = r.right = 0;
    r.s1 = r.s2 = 0.0f;
    r.z1 = key_at(lf, S, 2, n - 1); r.z0 = key_at(lf, S, 5, 0);
    r.y1 = key_at(lf, S, 1, n - 1); r.y0 = key_at(lf, S, 4, 0);
    r.x0 = key_at(lf, S, 3, 0);     r.x1 = key_at(lf, S, 0, n - 1);
}

struct Shape {
    const int32_t* l;
    const int32_t* m;
    const int32_t* r;
    const int32_t* left;    // first child, -1 for a leaf
    const int32_t* parent;
};

// The nodes [lv0, lv1) of one level: a leaf takes its triangle and its
// parent's cut flag (TD/Trixel.h:194-205); an interior node chooses its cut
// by the largest key span, strict `>` in the order x1, x0, y1, y0, z1, z0.
__global__ void k_level_nodes(const rt_leaf_aabb* __restrict__ lf, Lists S, Shape G, int64_t lv0, int64_t lv1,
                              rt_kd_node* __restrict__ nodes) {
    const int64_t id = lv0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= lv1) return;
    const int32_t l = G.l[id], r = G.r[id];
    rt_kd_node& nd = nodes[id];
    if (r == l) {
        nd.cut_flag = nodes[G.parent[id]].cut_flag;
        nd.is_leaf = 1;
        nd.left = -1;
        nd.right = -1;
        nd.tri_index = lf[S.at(0, l)].tri;
        return;
    }
    float best = key_at(lf, S, 0, r) - key_at(lf, S, 0, l);
    int cut = 0;
    const int order[5] = {3, 1, 4, 2, 5};
    for (int q = 0; q < 5; q++) {
        const int k = order[q];
        const float span = key_at(lf, S, k, r) - key_at(lf, S, k, l);
        if (span > best) { best = span; cut = k; }
    }
    nd.cut_flag = cut;
    nd.is_leaf = 0;
    nd.tri_index = -1;
    nd.left = G.left[id];
    nd.right = G.left[id] + 1;
}

__device__ __forceinline__ bool splits_here(const Shape& G, int32_t node, int64_t lv0, int64_t lv1) {
    return node >= lv0 && node < lv1 && G.l[node] != G.r[node];
}

// Which elements go left: positions l..m of the node's cut list.
__global__ void k_mark(Lists S, Shape G, const int32_t* __restrict__ posnode, const rt_kd_node* __restrict__ nodes,
                       int64_t lv0, int64_t lv1, uint8_t* __restrict__ inleft) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= S.n) return;
    const int32_t node = posnode[p];
    if (!splits_here(G, node, lv0, lv1)) return;
    inleft[S.at(nodes[node].cut_flag, p)] = p <= G.m[node] ? 1 : 0;
}

__global__ void k_flags(Lists S, Shape G, const int32_t* __restrict__ posnode, const uint8_t* __restrict__ inleft,
                        int64_t lv0, int64_t lv1, int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 6 * (int64_t)S.n) return;
    const int64_t p = i % S.n;
    const int32_t node = posnode[p];
    flags[i] = splits_here(G, node, lv0, lv1) ? (int32_t)inleft[S.L[i]] : 0;
}

// Stable partition of every list inside every splitting node's range
// (TD/Trixel.h:214-327): left elements to l.., right ones to m+1.., each in
// list order; positions outside the level's splitting ranges stay.
__global__ void k_scatter(Lists S, Shape G, const int32_t* __restrict__ posnode, const int32_t* __restrict__ flags,
                          const int32_t* __restrict__ scan, int64_t lv0, int64_t lv1, uint32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = S.n;
    if (i >= 6 * n) return;
    const int64_t k = i / n, p = i - k * n;
    const int32_t node = posnode[p];
    int64_t dst = p;
    if (splits_here(G, node, lv0, lv1)) {
        const int64_t l = G.l[node], m = G.m[node];
        const int64_t before = (int64_t)scan[i] - (int64_t)scan[k * n + l];  // left elements in [l, p)
        dst = flags[i] ? l + before : m + 1 + (p - l) - before;
    }
    out[k * n + dst] = S.L[i];
}

__global__ void k_descend(Shape G, int64_t n, int64_t lv0, int64_t lv1, int32_t* __restrict__ posnode) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int32_t node = posnode[p];
    if (!splits_here(G, node, lv0, lv1)) return;
    posnode[p] = p <= G.m[node] ? G.left[node] : G.left[node] + 1;
}

// A splitting node's children (TD/Trixel.h:329-376): boxes from the ends of
// their ranges in the partitioned lists, then the node's s1 (left child's
// max) and s2 (right child's min) on the cut axis.
__global__ void k_children(const rt_leaf_aabb* __restrict__ lf, Lists S, Shape G, int64_t lv0, int64_t lv1,
                           rt_kd_node* __restrict__ nodes) {
    const int64_t id = lv0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= lv1 || G.l[id] == G.r[id]) return;
    const int32_t cb = G.left[id];
    for (int br = 0; br < 2; br++) {
        rt_kd_node& c = nodes[cb + br];
        const int64_t nl = G.l[cb + br], nr = G.r[cb + br];
        c.parent = id;
        c.is_leaf = 0;
        c.tri_index = -1;
        c.left = c.right = 0;
        c.s1 = c.s2 = 0.0f;
        c.cut_flag = 0;
        c.x1 = key_at(lf, S, 0, nr); c.x0 = key_at(lf, S, 3, nl);
        c.y1 = key_at(lf, S, 1, nr); c.y0 = key_at(lf, S, 4, nl);
        c.z1 = key_at(lf, S, 2, nr); c.z0 = key_at(lf, S, 5, nl);
    }
    rt_kd_node& nd = nodes[id];
    const rt_kd_node& Lc = nodes[cb];
    const rt_kd_node& Rc = nodes[cb + 1];
    switch (nd.cut_flag) {
    case 0: case 3: nd.s2 = Rc.x0; nd.s1 = Lc.x1; break;
    case 1: case 4: nd.s2 = Rc.y0; nd.s1 = Lc.y1; break;
    default:        nd.s2 = Rc.z0; nd.s1 = Lc.z1; break;
    }
}

// node -> traversal ref: kLeafBit | triangle for a leaf, the record position
// for an interior node (ids = the interior nodes in record order).
__global__ void k_node_ref(const rt_kd_node* __restrict__ nodes, int64_t nnode, const int32_t* __restrict__ ids,
                           int64_t ninterior, uint32_t* __restrict__ ref) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ninterior) ref[ids[i]] = (uint32_t)i;
    if (i < nnode && nodes[i].is_leaf) ref[i] = kLeafBit | (uint32_t)nodes[i].tri_index;
}

unsigned blocks(int64_t n) { return (unsigned)((n + kBlk - 1) / kBlk); }

template <class T>
struct DevBuf {
    T* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int alloc(size_t count, const char* what) {
        hipError_t e = hipMalloc((void**)&p, sizeof(T) * (count ? count : 1));
        return e == hipSuccess ? RT_OK : fail(e == hipErrorOutOfMemory ? RT_ERR_NOMEM : RT_ERR_HIP, "%s: %s", what,
                                              hipGetErrorString(e));
    }
};

int hipck(hipError_t e, const char* what) {
    return e == hipSuccess ? RT_OK : fail(RT_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

}  // namespace

void kd_shape(uint32_t n, KdShape& out) {
    const int64_t nnode = 2 * (int64_t)n - 1;
    out.l.assign((size_t)nnode, 0);
    out.m.assign((size_t)nnode, 0);
    out.r.assign((size_t)nnode, 0);
    out.left.assign((size_t)nnode, -1);
    out.parent.assign((size_t)nnode, 0);
    out.level.assign(1, 0);
    out.l[0] = 0; out.r[0] = (int32_t)n - 1; out.m[0] = (int32_t)((n - 1) / 2);
    int64_t lv0 = 0, lv1 = 1, wr = 1;
    while (lv0 < lv1) {
        out.level.push_back(lv1);
        for (int64_t id = lv0; id < lv1; id++) {
            const int32_t l = out.l[(size_t)id], m = out.m[(size_t)id], r = out.r[(size_t)id];
            if (l == r) continue;
            out.left[(size_t)id] = (int32_t)wr;
            const int32_t cl[2] = {l, m + 1}, cr[2] = {m, r};
            for (int br = 0; br < 2; br++) {
                const size_t c = (size_t)(wr + br);
                out.l[c] = cl[br];
                out.r[c] = cr[br];
                out.m[c] = ((cr[br] - cl[br]) / 2) + cl[br];
                out.parent[c] = (int32_t)id;
            }
            wr += 2;
        }
        lv0 = lv1;
        lv1 = wr;
    }
    // level k = nodes [level[k], level[k+1]); the last entry is nnode
    out.height = (int32_t)out.level.size() - 2;
}

int kd_build_device(const rt_leaf_aabb* h_leafs, uint32_t n, const KdShape& G, rt_kd_node* d_nodes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int64_t nnode = 2 * (int64_t)n - 1;
    int rc;
    DevBuf<rt_leaf_aabb> lf;
    DevBuf<uint32_t> L0, L1, keys, keys2;
    DevBuf<int32_t> gl, gm, gr, gleft, gparent, posnode, flags, scan;
    DevBuf<uint8_t> inleft;
    if ((rc = lf.alloc(n, "kd gpu: leafs")) || (rc = L0.alloc(6 * (size_t)n, "kd gpu: lists")) ||
        (rc = L1.alloc(6 * (size_t)n, "kd gpu: lists")) || (rc = keys.alloc(n, "kd gpu: keys")) ||
        (rc = keys2.alloc(n, "kd gpu: keys")) || (rc = gl.alloc((size_t)nnode, "kd gpu: shape")) ||
        (rc = gm.alloc((size_t)nnode, "kd gpu: shape")) || (rc = gr.alloc((size_t)nnode, "kd gpu: shape")) ||
        (rc = gleft.alloc((size_t)nnode, "kd gpu: shape")) || (rc = gparent.alloc((size_t)nnode, "kd gpu: shape")) ||
        (rc = posnode.alloc(n, "kd gpu: posnode")) || (rc = flags.alloc(6 * (size_t)n, "kd gpu: flags")) ||
        (rc = scan.alloc(6 * (size_t)n, "kd gpu: scan")) || (rc = inleft.alloc(n, "kd gpu: inleft")))
        return rc;
    const size_t nb = sizeof(int32_t) * (size_t)nnode;
    if ((rc = hipck(hipMemcpyAsync(lf.p, h_leafs, sizeof(rt_leaf_aabb) * n, hipMemcpyHostToDevice, st), "H2D leafs")) ||
        (rc = hipck(hipMemcpyAsync(gl.p, G.l.data(), nb, hipMemcpyHostToDevice, st), "H2D shape")) ||
        (rc = hipck(hipMemcpyAsync(gm.p, G.m.data(), nb, hipMemcpyHostToDevice, st), "H2D shape")) ||
        (rc = hipck(hipMemcpyAsync(gr.p, G.r.data(), nb, hipMemcpyHostToDevice, st), "H2D shape")) ||
        (rc = hipck(hipMemcpyAsync(gleft.p, G.left.data(), nb, hipMemcpyHostToDevice, st), "H2D shape")) ||
        (rc = hipck(hipMemcpyAsync(gparent.p, G.parent.data(), nb, hipMemcpyHostToDevice, st), "H2D shape")) ||
        (rc = hipck(hipMemsetAsync(posnode.p, 0, sizeof(int32_t) * n, st), "memset posnode")))
        return rc;
    // the six sorted position lists (set_sorted_voxels, TD/Trixel.h:386-473)
    size_t sort_bytes = 0, scan_bytes = 0;
    if ((rc = hipck(rocprim::radix_sort_pairs(nullptr, sort_bytes, keys.p, keys2.p, L1.p, L0.p, n, 0, 32, st),
                    "radix sort size")) ||
        (rc = hipck(rocprim::exclusive_scan(nullptr, scan_bytes, flags.p, scan.p, 0, 6 * (size_t)n,
                                            rocprim::plus<int32_t>(), st), "scan size")))
        return rc;
    DevBuf<uint8_t> tmp;
    if ((rc = tmp.alloc(std::max(sort_bytes, scan_bytes), "kd gpu: temp"))) return rc;
    for (int k = 0; k < 6; k++) {
        k_sort_input<<<blocks(n), kBlk, 0, st>>>(lf.p, n, k, keys.p, L1.p);
        size_t b = sort_bytes;
        if ((rc = hipck(rocprim::radix_sort_pairs(tmp.p, b, keys.p, keys2.p, L1.p, L0.p + (size_t)k * n, n, 0, 32, st),
                        "radix sort")))
            return rc;
    }
    Shape S{gl.p, gm.p, gr.p, gleft.p, gparent.p};
    uint32_t* cur = L0.p;
    uint32_t* nxt = L1.p;
    k_root<<<1, 1, 0, st>>>(lf.p, Lists{cur, n}, d_nodes);
    const int64_t n6 = 6 * (int64_t)n;
    for (size_t lv = 0; lv + 1 < G.level.size(); lv++) {
        const int64_t lv0 = G.level[lv], lv1 = G.level[lv + 1];
        const Lists C{cur, n};
        k_level_nodes<<<blocks(lv1 - lv0), kBlk, 0, st>>>(lf.p, C, S, lv0, lv1, d_nodes);
        if (lv1 >= nnode) break;  // the last level is all leaves
        k_mark<<<blocks(n), kBlk, 0, st>>>(C, S, posnode.p, d_nodes, lv0, lv1, inleft.p);
        k_flags<<<blocks(n6), kBlk, 0, st>>>(C, S, posnode.p, inleft.p, lv0, lv1, flags.p);
        size_t b = scan_bytes;
        if ((rc = hipck(rocprim::exclusive_scan(tmp.p, b, flags.p, scan.p, 0, (size_t)n6, rocprim::plus<int32_t>(), st),
                        "scan")))
            return rc;
        k_scatter<<<blocks(n6), kBlk, 0, st>>>(C, S, posnode.p, flags.p, scan.p, lv0, lv1, nxt);
        k_descend<<<blocks(n), kBlk, 0, st>>>(S, n, lv0, lv1, posnode.p);
        k_children<<<blocks(lv1 - lv0), kBlk, 0, st>>>(lf.p, Lists{nxt, n}, S, lv0, lv1, d_nodes);
        std::swap(cur, nxt);
    }
    if ((rc = hipck(hipGetLastError(), "kd gpu launch"))) return rc;
    return hipck(hipStreamSynchronize(st), "kd gpu sync");
}

int launch_node_ref(const rt_kd_node* d_nodes, int64_t nnode, const int32_t* d_ids, int64_t ninterior,
                    uint32_t* d_ref, void* stream) {
    if (nnode == 0) return RT_OK;
    k_node_ref<<<blocks(nnode), kBlk, 0, (hipStream_t)stream>>>(d_nodes, nnode, d_ids, ninterior, d_ref);
    return hipck(hipGetLastError(), "k_node_ref launch");
}

}  // namespace rt
