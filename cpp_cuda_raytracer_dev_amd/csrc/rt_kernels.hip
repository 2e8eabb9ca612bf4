// rt_kernels.hip -- the launchers of the gfx950 kernels (rt_kernels_impl.h).
// The KD kernels' instances live in rt_kd_dispatch.hip, compiled once per
// (translated, write-hit, count) combination (build.py).
#include "rt_kernels_impl.h"

namespace rt {

// rt_kd_dispatch.hip: the KD kernel of one (translated, write-hit, count) combination.
#define RT_KD_DECL(t, h, c) TraceFn kd_kernel_##t##h##c(int version, int rays, int shadow, bool coarse);
RT_KD_DECL(0, 0, 0) RT_KD_DECL(0, 0, 1) RT_KD_DECL(0, 1, 0) RT_KD_DECL(0, 1, 1)
RT_KD_DECL(1, 0, 0) RT_KD_DECL(1, 0, 1) RT_KD_DECL(1, 1, 0) RT_KD_DECL(1, 1, 1)
#undef RT_KD_DECL

int launch_tri_world(const float* points9, const float* rad3, uint32_t ntri, float4* tri_world,
                     float4* shade, void* stream) {
    if (ntri == 0) return RT_OK;
    k_tri_world<<<(ntri + 255) / 256, 256, 0, (hipStream_t)stream>>>(points9, rad3, ntri, tri_world, shade);
    return check_launch<void>("k_tri_world");
}

int launch_cam_tri(const float4* tri_world, uint32_t ntri, const float pos[3], float4* trec,
                   void* stream) {
    if (ntri == 0) return RT_OK;
    k_cam_tri<<<(ntri + 255) / 256, 256, 0, (hipStream_t)stream>>>(tri_world, ntri, pos[0], pos[1], pos[2], trec);
    return check_launch<void>("k_cam_tri");
}

int launch_cam_nodes(const rt_kd_node* nodes, const int32_t* ids, const uint32_t* node_ref,
                     int64_t ninterior, const float pos[3], float4* inode, int32_t* flags, void* stream) {
    if (ninterior == 0) return RT_OK;
    k_cam_nodes<<<(unsigned)((ninterior + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        nodes, ids, node_ref, ninterior, pos[0], pos[1], pos[2], inode, flags);
    return check_launch<void>("k_cam_nodes");
}


int launch_pair_tri(const float4* trec, uint32_t ntri, float4* tpair, void* stream) {
    if (ntri == 0) return RT_OK;
    const uint32_t npair = (ntri + 1) >> 1;
    k_pair_tri<<<(npair + 255) / 256, 256, 0, (hipStream_t)stream>>>(trec, ntri, tpair);
    return check_launch<void>("k_pair_tri");
}

int launch_trace(const TraceParams& p, uint32_t mode, uint32_t flags, int kernel_version, void* stream, int part) {
    hipStream_t s = (hipStream_t)stream;
    const bool wh = (flags & RT_FLAG_WRITE_HIT) != 0, cnt = (flags & RT_FLAG_COUNT) != 0;
    const unsigned fine = (unsigned)(p.tiles_x * p.block_rows);
    // waves per block = (tile_w / 8) * (tile_h / (rays / 8))
    const unsigned threads = (unsigned)((p.tile_w / 8) * (p.tile_h / (p.rays / 8)) * 64);
    if (mode == RT_MODE_FLAT) {
        if (fine == 0) return RT_OK;
        if (p.flat_key && !cnt) {  // the chunked form: the chunks, then the shading
            k_flat_chunk<<<fine * (unsigned)p.flat_chunks, threads, 0, s>>>(p);
            int rc = check_launch<void>("k_flat_chunk");
            if (rc) return rc;
            (wh ? k_flat_shade<true> : k_flat_shade<false>)<<<fine, threads, 0, s>>>(p);
            return check_launch<void>("k_flat_shade");
        }
        // one pass (form 9, and counting renders: the accept counter counts
        // updates of the running minimum in index order)
        TraceFn fn = wh ? (cnt ? k_trace_flat<true, true> : k_trace_flat<true, false>)
                        : (cnt ? k_trace_flat<false, true> : k_trace_flat<false, false>);
        fn<<<fine, threads, 0, s>>>(p);
        return check_launch<void>("k_trace_flat");
    }
    const bool tr = p.xf[3] != 0.0f || p.xf[7] != 0.0f || p.xf[11] != 0.0f;
    const int v = kernel_version, r = p.rays;
    const int sh = (flags & RT_FLAG_SHADOW) ? p.any_order : -1;  // kernel 3 only (checked by the caller)
    for (int pass = 0; pass < 2; pass++) {
        // the coarse groups first, then the fine tiles (or just one of them)
        const bool coarse = pass == 0;
        if ((coarse && part == kPartFine) || (!coarse && part == kPartCoarse)) continue;
        unsigned grid = coarse ? (unsigned)p.coarse_blocks : fine_grid_blocks(p);
        if (grid == 0) continue;
        TraceFn fn;
        if (tr) fn = wh ? (cnt ? kd_kernel_111(v, r, sh, coarse) : kd_kernel_110(v, r, sh, coarse))
                        : (cnt ? kd_kernel_101(v, r, sh, coarse) : kd_kernel_100(v, r, sh, coarse));
        else fn = wh ? (cnt ? kd_kernel_011(v, r, sh, coarse) : kd_kernel_010(v, r, sh, coarse))
                     : (cnt ? kd_kernel_001(v, r, sh, coarse) : kd_kernel_000(v, r, sh, coarse));
        if (!coarse && p.pf_frames > 0) grid = (unsigned)p.pf_blocks * (unsigned)p.pf_frames;  // a multi-frame launch, frame-major
        fn<<<grid, coarse ? 128u : threads, 0, s>>>(p);
        int rc = check_launch<void>(coarse ? "k_coarse_kd3" : "k_trace_kd");
        if (rc) return rc;
    }
    return RT_OK;
}

int launch_unpack(int32_t w, int32_t h, int32_t nranks, const uint32_t* gathered, uint32_t* frame,
                  void* stream) {
    const int32_t nbands = (h + kTileH - 1) / kTileH;
    const int32_t slots = (nbands + nranks - 1) / nranks;
    if ((int64_t)w * h == 0) return RT_OK;
    const int32_t vec = (w & 3) == 0 && ((uintptr_t)gathered & 15) == 0 && ((uintptr_t)frame & 15) == 0;
    const int32_t per_row = vec ? (w >> 2) : w;
    const dim3 grid((unsigned)((per_row + 255) / 256), (unsigned)h);
    k_unpack<<<grid, 256, 0, (hipStream_t)stream>>>(w, h, nranks, slots, vec, gathered, frame);
    return check_launch<void>("k_unpack");
}

int launch_pack_rect(int32_t w, int32_t h, int32_t nranks, int32_t rank, const int32_t rect[4],
                     const uint32_t* local, uint32_t* out, void* stream) {
    int32_t s0, s1;
    rect_slots(rect[2], rect[3], nranks, rank, s0, s1);
    const int32_t cw = rect[1] - rect[0];
    if (cw <= 0 || s1 <= s0) return RT_OK;
    (void)h;
    const dim3 grid((unsigned)((cw + 255) / 256), (unsigned)((s1 - s0) * kTileH));
    k_pack_rect<<<grid, 256, 0, (hipStream_t)stream>>>(w, rect[0], cw, s0, local, out);
    return check_launch<void>("k_pack_rect");
}

int launch_unpack_rect(int32_t w, int32_t h, int32_t nranks, const int32_t rect[4], const uint32_t* local0,
                       const uint32_t* peers, uint32_t* frame, void* stream, bool rect_only) {
    if ((int64_t)w * h == 0) return RT_OK;
    const int32_t vec = ((w & 3) == 0 && ((uintptr_t)frame & 15) == 0) ? 4 : 1;
    int32_t y0 = 0, xa = 0, rows = h, cols = w;
    if (rect_only) {
        if (rect[0] >= rect[1] || rect[2] >= rect[3]) return RT_OK;
        y0 = rect[2] * kTileH;
        rows = std::min(rect[3] * kTileH, h) - y0;
        xa = rect[0] - rect[0] % vec;
        cols = rect[1] - xa;
    }
    const int32_t per_row = (cols + vec - 1) / vec;
    // the rectangle alone runs beside the next frames' renders: 8 rows per
    // block keeps its dispatch short (one block per row took 18 us there)
    const int32_t rpb = rect_only ? 8 : 1;
    const dim3 grid((unsigned)((per_row + 255) / 256), (unsigned)((rows + rpb - 1) / rpb));
    k_unpack_rect<<<grid, 256, 0, (hipStream_t)stream>>>(w, nranks, rect[0], rect[1], rect[2], rect[3], vec, y0, xa,
                                                         rows, rpb, local0, peers, frame);
    return check_launch<void>("k_unpack_rect");
}

}  // namespace rt
