// rccl_shim.cpp -- TEST-ONLY stand-in for librccl.so.1.
//
// Lets the library's real N > 1 frame gather (csrc/comm.cpp: rank 0's
// ncclRecv loop, the peers' pack + ncclSend, rank 0's direct-path assembly)
// run with N ranks inside ONE process on ONE GPU: the ranks are threads, each
// with its own rt_camera, rt_comm and streams, all on device 0.  It is loaded
// through RT_RCCL_LIB (comm.cpp's dlopen override) by tests/shim_ranks.py and
// nowhere else; the product never links or loads it.
//
// Semantics are those of point-to-point NCCL inside a group:
//   * ncclCommInitRank registers the rank under its unique id (no blocking);
//   * send / recv calls between ncclGroupStart / ncclGroupEnd are collected and
//     executed at the outermost ncclGroupEnd (a call outside a group is a group
//     of one);
//   * a send records a "ready" event on its stream and posts (buffer, bytes,
//     event) on the (src, dst) queue; the matching recv -- the oldest posting on
//     that queue, as NCCL matches them in call order -- makes its stream wait
//     for "ready", copies the bytes device to device on its stream and records
//     a "done" event; the sender's stream then waits for "done", so a send
//     completes, in stream order, once the data has left its buffer.
//   The rendezvous blocks the calling host threads (a recv waits for the
//   matching post, a send for the recv's copy to be enqueued); frame loops
//   issue their gathers in frame order on every rank, so they pair up.
//   A recv whose byte count differs from the send's fails (ncclInvalidUsage),
//   as a real truncated receive would be an error.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace {

typedef int nres_t;
constexpr nres_t kOk = 0, kHipError = 1, kInvalidArgument = 4, kInvalidUsage = 5;
constexpr int kIdBytes = 128;

struct Msg {
    const void* src = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr, done = nullptr;
    bool replied = false;
    nres_t status = kOk;
};

struct Group {
    int nranks = 0;
    int live = 0;  // comms not yet destroyed
    std::mutex m;
    std::condition_variable cv;
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> q;  // (src, dst) -> posted sends
    std::vector<hipEvent_t> retired;                                     // destroyed after the last comm
};

struct Comm {
    Group* g;
    int rank, nranks;
};

struct Op {
    bool send;
    const void* sbuf;
    void* rbuf;
    size_t bytes;
    int peer;
    Comm* c;
    hipStream_t s;
};

std::mutex g_m;
std::map<std::string, Group*> g_groups;
std::atomic<uint64_t> g_next{1};
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

size_t type_bytes(int t) {
    switch (t) {
    case 0: case 1: return 1;            // int8, uint8
    case 2: case 3: case 7: return 4;    // int32, uint32, float32
    case 4: case 5: case 8: return 8;    // int64, uint64, float64
    case 6: case 9: return 2;            // float16, bfloat16
    default: return 0;
    }
}

nres_t hip_ok(hipError_t e) { return e == hipSuccess ? kOk : kHipError; }

nres_t run_group(std::vector<Op>& ops) {
    nres_t rc = kOk;
    std::vector<std::shared_ptr<Msg>> posted(ops.size());
    // 1. every send posts its buffer behind a "ready" event
    for (size_t i = 0; i < ops.size() && rc == kOk; i++) {
        Op& o = ops[i];
        if (!o.send) continue;
        auto m = std::make_shared<Msg>();
        m->src = o.sbuf;
        m->bytes = o.bytes;
        if ((rc = hip_ok(hipEventCreateWithFlags(&m->ready, hipEventDisableTiming)))) break;
        if ((rc = hip_ok(hipEventRecord(m->ready, o.s)))) break;
        Group* g = o.c->g;
        {
            std::lock_guard<std::mutex> lk(g->m);
            g->q[{o.c->rank, o.peer}].push_back(m);
        }
        g->cv.notify_all();
        posted[i] = m;
    }
    // 2. every recv takes the oldest matching posting and copies it
    for (size_t i = 0; i < ops.size() && rc == kOk; i++) {
        Op& o = ops[i];
        if (o.send) continue;
        Group* g = o.c->g;
        std::shared_ptr<Msg> m;
        {
            std::unique_lock<std::mutex> lk(g->m);
            auto& dq = g->q[{o.peer, o.c->rank}];
            g->cv.wait(lk, [&] { return !dq.empty(); });
            m = dq.front();
            dq.pop_front();
        }
        nres_t st = m->bytes == o.bytes ? kOk : kInvalidUsage;
        if (st != kOk)
            fprintf(stderr, "rccl_shim: recv of %zu bytes by rank %d from %d matched a send of %zu bytes\n", o.bytes,
                    o.c->rank, o.peer, m->bytes);
        if (st == kOk) st = hip_ok(hipStreamWaitEvent(o.s, m->ready, 0));
        if (st == kOk && o.bytes) st = hip_ok(hipMemcpyAsync(o.rbuf, m->src, o.bytes, hipMemcpyDeviceToDevice, o.s));
        if (st == kOk) st = hip_ok(hipEventCreateWithFlags(&m->done, hipEventDisableTiming));
        if (st == kOk) st = hip_ok(hipEventRecord(m->done, o.s));
        {
            std::lock_guard<std::mutex> lk(g->m);
            m->status = st;
            m->replied = true;
        }
        g->cv.notify_all();
        rc = st;
    }
    // 3. every send's stream waits until its data has been copied out
    for (size_t i = 0; i < ops.size(); i++) {
        Op& o = ops[i];
        if (!o.send || !posted[i]) continue;
        auto& m = posted[i];
        Group* g = o.c->g;
        {
            std::unique_lock<std::mutex> lk(g->m);
            g->cv.wait(lk, [&] { return m->replied; });
            g->retired.push_back(m->ready);
            if (m->done) g->retired.push_back(m->done);
        }
        if (rc == kOk) rc = m->status;
        if (rc == kOk && m->done) rc = hip_ok(hipStreamWaitEvent(o.s, m->done, 0));
    }
    return rc;
}

nres_t enqueue(const Op& o) {
    if (!o.c || o.peer < 0 || o.peer >= o.c->nranks || o.peer == o.c->rank) return kInvalidArgument;
    t_ops.push_back(o);
    if (t_depth > 0) return kOk;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_group(ops);
}

}  // namespace

extern "C" {

nres_t ncclGetUniqueId(void* id) {
    if (!id) return kInvalidArgument;
    memset(id, 0, kIdBytes);
    snprintf((char*)id, kIdBytes, "rt-rccl-shim-%d-%llu", (int)getpid(), (unsigned long long)g_next++);
    return kOk;
}

// ncclUniqueId is passed by value (128 bytes): the same layout as a struct of
// that size in the caller's ABI
struct shim_uid {
    char internal[kIdBytes];
};

nres_t ncclCommInitRank(void** comm, int nranks, shim_uid id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return kInvalidArgument;
    std::lock_guard<std::mutex> lk(g_m);
    Group*& g = g_groups[std::string(id.internal, strnlen(id.internal, kIdBytes))];
    if (!g) {
        g = new Group;
        g->nranks = nranks;
    }
    if (g->nranks != nranks) return kInvalidUsage;
    g->live++;
    *comm = new Comm{g, rank, nranks};
    return kOk;
}

nres_t ncclCommDestroy(void* comm) {
    Comm* c = (Comm*)comm;
    if (!c) return kInvalidArgument;
    Group* g = c->g;
    bool last;
    {
        std::lock_guard<std::mutex> lk(g_m);
        last = --g->live == 0;
    }
    if (last) {
        (void)hipDeviceSynchronize();  // every copy and wait of the group has run
        for (hipEvent_t e : g->retired) (void)hipEventDestroy(e);
        g->retired.clear();
    }
    delete c;
    return kOk;
}

nres_t ncclGroupStart(void) {
    t_depth++;
    return kOk;
}

nres_t ncclGroupEnd(void) {
    if (t_depth <= 0) return kInvalidUsage;
    if (--t_depth > 0) return kOk;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_group(ops);
}

nres_t ncclSend(const void* buf, size_t count, int dtype, int peer, void* comm, hipStream_t s) {
    const size_t b = type_bytes(dtype);
    if (!b) return kInvalidArgument;
    return enqueue(Op{true, buf, nullptr, count * b, peer, (Comm*)comm, s});
}

nres_t ncclRecv(void* buf, size_t count, int dtype, int peer, void* comm, hipStream_t s) {
    const size_t b = type_bytes(dtype);
    if (!b) return kInvalidArgument;
    return enqueue(Op{false, nullptr, buf, count * b, peer, (Comm*)comm, s});
}

const char* ncclGetErrorString(nres_t r) {
    switch (r) {
    case kOk: return "no error (rccl_shim)";
    case kHipError: return "HIP call failed (rccl_shim)";
    case kInvalidArgument: return "invalid argument (rccl_shim)";
    case kInvalidUsage: return "invalid usage: send/recv sizes differ (rccl_shim)";
    default: return "unknown error (rccl_shim)";
    }
}

}  // extern "C"
