// comm.cpp -- the multi-GPU frame gather over RCCL.
//
// The reference is single-GPU (cudaSetDevice(0), TD/Trixel.cu:213); this is
// new.  Each rank renders its interleaved 8-row bands into a packed buffer
// (rt_render_into with an rt_tile); one rt_comm_gather_frame call then moves
// every peer's part of the frame to rank 0 over xGMI and assembles the frame
// there, all stream-ordered on the caller's stream.  Only the rectangle
// rt_frame_rect names travels: outside it every pixel is provably background.
//   rank != 0: k_pack_rect(local -> scratch); ncclSend(scratch -> 0)
//   rank == 0: ncclRecv(scratch + off_r <- r) for r = 1..N-1 (one group);
//              k_unpack_rect(local, scratch, background -> frame)
// i.e. N-1 point-to-point transfers, one xGMI link per peer, no ring.  The
// host cost is a handful of enqueue calls, so a frame loop (or a captured
// graph of frames) is not bound by the collective's Python path.
//
// RCCL is resolved at run time (dlopen of librccl.so.1): a process that
// already holds PyTorch's RCCL gets that same library (dlopen matches the
// soname), otherwise ROCm's; the environment variable RT_RCCL_LIB names
// another library with the same entry points (the test-only shim of
// tests/rccl_shim, which runs N ranks as threads of one process).  Nothing here runs without a GPU, and the
// library loads on machines without RCCL (rt_comm_* then fail loudly).
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <type_traits>

#include "rt_internal.h"

using namespace rt;

namespace {

// The slice of rccl.h this file calls (types by value, as the ABI has them).
typedef int nres_t;  // ncclResult_t; 0 = ncclSuccess
typedef void* ncomm_t;
struct nuid_t {
    char internal[RT_COMM_ID_BYTES];
};
constexpr int kNcclUint32 = 3;  // ncclDataType_t ncclUint32

struct Rccl {
    void* so = nullptr;
    nres_t (*get_unique_id)(nuid_t*) = nullptr;
    nres_t (*comm_init_rank)(ncomm_t*, int, nuid_t, int) = nullptr;
    nres_t (*comm_destroy)(ncomm_t) = nullptr;
    nres_t (*send)(const void*, size_t, int, int, ncomm_t, hipStream_t) = nullptr;
    nres_t (*recv)(void*, size_t, int, int, ncomm_t, hipStream_t) = nullptr;
    nres_t (*group_start)() = nullptr;
    nres_t (*group_end)() = nullptr;
    const char* (*error_string)(nres_t) = nullptr;
    bool ok = false;
};

Rccl g_rccl;
std::once_flag g_rccl_once;

const Rccl* rccl() {
    std::call_once(g_rccl_once, [] {
        const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        // RT_RCCL_LIB: an explicit library instead (tests/rccl_shim: N ranks
        // as threads of one process on one GPU); it must load, no fallback
        const char* over = getenv("RT_RCCL_LIB");
        void* so = over && *over ? dlopen(over, RTLD_NOW | RTLD_LOCAL) : dlopen(names[0], RTLD_NOW | RTLD_NOLOAD);
        for (int k = 0; !so && !(over && *over) && k < 3; ++k) so = dlopen(names[k], RTLD_NOW | RTLD_LOCAL);
        if (!so) return;
        Rccl r;
        r.so = so;
        bool all = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(so, name));
            all = all && fp;
        };
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.comm_init_rank, "ncclCommInitRank");
        sym(r.comm_destroy, "ncclCommDestroy");
        sym(r.send, "ncclSend");
        sym(r.recv, "ncclRecv");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.error_string, "ncclGetErrorString");
        r.ok = all;
        g_rccl = r;
    });
    return g_rccl.ok ? &g_rccl : nullptr;
}

int nccl_check(const Rccl* r, nres_t e, const char* what) {
    if (e == 0) return RT_OK;
    return fail(RT_ERR_COMM, "%s: %s", what, r->error_string ? r->error_string(e) : "rccl error");
}

struct Guard {
    int prev = -1;
    bool ok = false;
    explicit Guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~Guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct rt_comm {
    int device = 0;
    int nranks = 1;
    int rank = 0;
    ncomm_t comm = nullptr;
};

extern "C" int rt_comm_available(void) { return rccl() ? 1 : 0; }

extern "C" int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]) {
    if (!id) return fail(RT_ERR_INVALID, "rt_comm_unique_id: null");
    const Rccl* r = rccl();
    if (!r) return fail(RT_ERR_COMM, "rt_comm_unique_id: librccl.so.1 not found or incomplete");
    nuid_t u;
    int rc = nccl_check(r, r->get_unique_id(&u), "ncclGetUniqueId");
    if (rc) return rc;
    memcpy(id, u.internal, RT_COMM_ID_BYTES);
    return RT_OK;
}

extern "C" int rt_comm_create(int device, int32_t nranks, int32_t rank, const uint8_t id[RT_COMM_ID_BYTES],
                              rt_comm** out) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(RT_ERR_INVALID, "rt_comm_create: bad argument (rank %d of %d)", rank, nranks);
    *out = nullptr;
    const Rccl* r = rccl();
    if (!r) return fail(RT_ERR_COMM, "rt_comm_create: librccl.so.1 not found or incomplete");
    Guard g(device);
    if (!g.ok) return fail(RT_ERR_HIP, "rt_comm_create: hipSetDevice(%d) failed", device);
    nuid_t u;
    memcpy(u.internal, id, RT_COMM_ID_BYTES);
    ncomm_t comm = nullptr;
    int rc = nccl_check(r, r->comm_init_rank(&comm, nranks, u, rank), "ncclCommInitRank");
    if (rc) return rc;
    rt_comm* c = new rt_comm;
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    c->comm = comm;
    *out = c;
    return RT_OK;
}

extern "C" int rt_comm_gather_frame(rt_comm* c, rt_camera* cam, const float* xform, uint32_t mode,
                                    const uint32_t* d_local, uint32_t* d_scratch, uint32_t* d_frame, void* stream) {
    return rt::comm_gather_frame(c, cam, xform, mode, d_local, d_scratch, d_frame, stream, false, nullptr);
}

int rt::comm_gather_frame(rt_comm* c, rt_camera* cam, const float* xform, uint32_t mode, const uint32_t* d_local,
                          uint32_t* d_scratch, uint32_t* d_frame, void* stream, bool rect_only, int32_t rect_out[4]) {
    if (!c || !cam || !d_local) return fail(RT_ERR_INVALID, "rt_comm_gather_frame: bad argument");
    if ((c->rank == 0 && !d_frame) || (c->nranks > 1 && !d_scratch))
        return fail(RT_ERR_INVALID, "rt_comm_gather_frame: missing scratch or frame buffer");
    int32_t w, h, depth;
    int rc;
    if ((rc = rt_camera_info(cam, &w, &h, &depth))) return rc;
    // the part of the frame that is not provably background: the same on
    // every rank (same camera, transform and options), so sizes need no
    // exchange
    int32_t rect[4];
    if ((rc = rt_frame_rect(cam, xform, mode, c->nranks, rect))) return rc;
    if (rect_out) memcpy(rect_out, rect, sizeof rect);
    const Rccl* r = rccl();
    Guard g(c->device);
    if (!g.ok) return fail(RT_ERR_HIP, "rt_comm_gather_frame: hipSetDevice(%d) failed", c->device);
    hipStream_t s = (hipStream_t)stream;
    if (c->rank == 0) {
        if (c->nranks > 1) {
            if ((rc = nccl_check(r, r->group_start(), "ncclGroupStart"))) return rc;
            int64_t off = 0;
            for (int p = 1; p < c->nranks && !rc; ++p) {
                const int64_t n = rt_rect_pixels(w, h, c->nranks, p, rect);
                if (n > 0) rc = nccl_check(r, r->recv(d_scratch + off, (size_t)n, kNcclUint32, p, c->comm, s), "ncclRecv");
                off += n;
            }
            const nres_t e = r->group_end();
            if (rc) return rc;
            if ((rc = nccl_check(r, e, "ncclGroupEnd"))) return rc;
        }
        // d_local == d_frame: rank 0 rendered its bands into the frame itself
        // (RT_FLAG_FRAME_OUT), so the assembly leaves them alone
        const bool own_in_frame = d_local == d_frame;
        if (own_in_frame && c->nranks == 1) return RT_OK;
        return launch_unpack_rect(w, h, c->nranks, rect, own_in_frame ? nullptr : d_local, d_scratch, d_frame, stream,
                                  rect_only);
    }
    const int64_t n = rt_rect_pixels(w, h, c->nranks, c->rank, rect);
    if (n <= 0) return RT_OK;
    if ((rc = rt_pack_rect(c->device, w, h, c->nranks, c->rank, rect, d_local, d_scratch, stream))) return rc;
    if ((rc = nccl_check(r, r->group_start(), "ncclGroupStart"))) return rc;
    rc = nccl_check(r, r->send(d_scratch, (size_t)n, kNcclUint32, 0, c->comm, s), "ncclSend");
    const nres_t e = r->group_end();
    if (rc) return rc;
    return nccl_check(r, e, "ncclGroupEnd");
}

extern "C" int rt_comm_info(const rt_comm* c, int32_t* nranks, int32_t* rank) {
    if (!c) return fail(RT_ERR_INVALID, "rt_comm_info: null");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return RT_OK;
}

extern "C" void rt_comm_destroy(rt_comm* c) {
    if (!c) return;
    const Rccl* r = rccl();
    if (r && c->comm) {
        Guard g(c->device);
        (void)r->comm_destroy(c->comm);
    }
    delete c;
}
