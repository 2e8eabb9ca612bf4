// scene_host.cpp -- host-side scene construction behind the C ABI:
// PLY input, the KD-tree builder and the camera basis.
//
// These are the producers of the hot path's inputs (SURVEY.md §8a rows a1,
// a11).  They reproduce the reference's results exactly (tests compare them
// with the oracle) but are organised for speed: the six merge sorts become
// stable radix sorts with the merge sort's tie order, and every level's
// partitions run as chunked count / scan / scatter passes on a thread pool
// (sibling ranges are disjoint; a big node's range is cut into chunks).
#include <math.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "rt_internal.h"

namespace rt {

static thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

namespace {

// Runs body(i) for i in [0, n) on up to `threads` std::threads.
template <class F>
void parallel_for(int64_t n, int threads, F&& body) {
    if (n <= 0) return;
    if (threads <= 1 || n == 1) {
        for (int64_t i = 0; i < n; i++) body(i);
        return;
    }
    std::atomic<int64_t> next{0};
    int t = (int)std::min<int64_t>(threads, n);
    std::vector<std::thread> pool;
    pool.reserve(t);
    for (int k = 0; k < t; k++)
        pool.emplace_back([&] {
            for (int64_t i; (i = next.fetch_add(1)) < n;) body(i);
        });
    for (auto& th : pool) th.join();
}

// nthreads <= 0: the CPUs this process may run on (its affinity mask, and
// OMP_NUM_THREADS when set lower), at most 64.  hardware_concurrency() counts
// the whole machine, which oversubscribes a container's CPU share.
int resolve_threads(int nthreads) {
    if (nthreads > 0) return nthreads;
    unsigned hc = std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) {
        const int c = CPU_COUNT(&set);
        if (c > 0) hc = std::min(hc ? hc : (unsigned)c, (unsigned)c);
    }
    if (const char* e = getenv("OMP_NUM_THREADS")) {
        const int v = atoi(e);
        if (v > 0) hc = std::min(hc ? hc : (unsigned)v, (unsigned)v);
    }
    return hc ? (int)std::min(hc, 64u) : 4;
}

// ------------------------------------------------------------- PLY input

// windows.h min/max as used by TD/read_ply.cpp:82-89,104-111,128-135 (order matters only
// for the sign of zero, which is kept identical anyway).
inline float wmin(float a, float b) { return (a < b) ? a : b; }
inline float wmax(float a, float b) { return (a > b) ? a : b; }

void aabb3(rt_leaf_aabb& lf, const float* a, const float* b, const float* c) {
    lf.x0 = wmin(a[0], wmin(b[0], c[0])); lf.x1 = wmax(a[0], wmax(b[0], c[0]));
    lf.y0 = wmin(a[1], wmin(b[1], c[1])); lf.y1 = wmax(a[1], wmax(b[1], c[1]));
    lf.z0 = wmin(a[2], wmin(b[2], c[2])); lf.z1 = wmax(a[2], wmax(b[2], c[2]));
}

struct Cursor {
    const char* p;
    const char* end;
    bool line(std::string& out) {
        out.clear();
        if (p >= end) return false;
        while (p < end && *p != '\n') {
            if (*p != '\r') out.push_back(*p);
            p++;
        }
        if (p < end) p++;
        return true;
    }
};

bool is_count_line(const std::string& s) {
    size_t i = 0;
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) i++;
    size_t d = i;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++;
    if (i == d) return false;
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) i++;
    return i == s.size();
}

}  // namespace
}  // namespace rt

using namespace rt;

extern "C" void rt_host_free(void* p) { free(p); }

extern "C" int rt_mesh_assemble(const float* verts, int64_t nvert, const int32_t* arity,
                                const int32_t* idx, int64_t nface, float** points9,
                                uint32_t* ntri_out, rt_leaf_aabb** leafs_out) {
    if (!points9 || !ntri_out || !leafs_out || (nface > 0 && (!arity || !idx || !verts)))
        return fail(RT_ERR_INVALID, "rt_mesh_assemble: null argument");
    int64_t ntri = 0;
    for (int64_t f = 0; f < nface; f++) {
        if (arity[f] == 3) ntri += 1;
        else if (arity[f] == 4) ntri += 2;
        else return fail(RT_ERR_INVALID, "rt_mesh_assemble: face %lld has arity %d", (long long)f, arity[f]);
    }
    if (ntri >= (int64_t)kLeafBit) return fail(RT_ERR_INVALID, "rt_mesh_assemble: too many triangles");
    float* pts = (float*)malloc(sizeof(float) * 9 * (size_t)std::max<int64_t>(ntri, 1));
    rt_leaf_aabb* lf = (rt_leaf_aabb*)malloc(sizeof(rt_leaf_aabb) * (size_t)std::max<int64_t>(ntri, 1));
    if (!pts || !lf) { free(pts); free(lf); return fail(RT_ERR_NOMEM, "rt_mesh_assemble: out of memory"); }
    int64_t t = 0, k = 0;
    auto put = [&](int64_t tri, int slot, const float* v) {
        float* d = pts + 9 * tri + 3 * slot;
        d[0] = v[0]; d[1] = v[1]; d[2] = v[2];
    };
    for (int64_t f = 0; f < nface; f++) {
        const int a = arity[f];
        for (int j = 0; j < a; j++)
            if (idx[k + j] < 0 || idx[k + j] >= nvert) {
                free(pts); free(lf);
                return fail(RT_ERR_INVALID, "rt_mesh_assemble: face %lld index out of range", (long long)f);
            }
        if (a == 4) {  // TD/read_ply.cpp:70-125: ABCD -> (A,B,C), (A,C,D)
            const float* A = verts + 3 * (int64_t)idx[k];
            const float* B = verts + 3 * (int64_t)idx[k + 1];
            const float* Cv = verts + 3 * (int64_t)idx[k + 2];
            const float* D = verts + 3 * (int64_t)idx[k + 3];
            aabb3(lf[t], A, B, Cv); lf[t].tri = t;
            put(t, 0, A); put(t, 1, B); put(t, 2, Cv); t++;
            aabb3(lf[t], A, D, Cv); lf[t].tri = t;
            put(t, 0, A); put(t, 1, Cv); put(t, 2, D); t++;
        } else {       // TD/read_ply.cpp:127-149: P1P2P3 stored as (P3,P1,P2)
            const float* P1 = verts + 3 * (int64_t)idx[k];
            const float* P2 = verts + 3 * (int64_t)idx[k + 1];
            const float* P3 = verts + 3 * (int64_t)idx[k + 2];
            aabb3(lf[t], P1, P2, P3); lf[t].tri = t;
            put(t, 0, P3); put(t, 1, P1); put(t, 2, P2); t++;
        }
        k += a;
    }
    *points9 = pts;
    *leafs_out = lf;
    *ntri_out = (uint32_t)ntri;
    return RT_OK;
}

namespace rt {
namespace {

// ---- PLY header (TD/read_ply.cpp:19-44, extended with property lists) ----

enum PlyType { kNone = 0, kI8, kU8, kI16, kU16, kI32, kU32, kF32, kF64 };

PlyType ply_type(const char* t) {
    static const struct { const char* n; PlyType t; } names[] = {
        {"char", kI8}, {"int8", kI8}, {"uchar", kU8}, {"uint8", kU8}, {"short", kI16}, {"int16", kI16},
        {"ushort", kU16}, {"uint16", kU16}, {"int", kI32}, {"int32", kI32}, {"uint", kU32}, {"uint32", kU32},
        {"float", kF32}, {"float32", kF32}, {"double", kF64}, {"float64", kF64}};
    for (const auto& e : names)
        if (!strcmp(t, e.n)) return e.t;
    return kNone;
}

int ply_size(PlyType t) {
    switch (t) {
    case kI8: case kU8: return 1;
    case kI16: case kU16: return 2;
    case kI32: case kU32: case kF32: return 4;
    case kF64: return 8;
    default: return 0;
    }
}

// Little-endian scalar of type t at p, as a double (exact for every type).
double ply_get(const unsigned char* p, PlyType t) {
    switch (t) {
    case kI8: return (double)(int8_t)p[0];
    case kU8: return (double)p[0];
    case kI16: { int16_t v; memcpy(&v, p, 2); return v; }
    case kU16: { uint16_t v; memcpy(&v, p, 2); return v; }
    case kI32: { int32_t v; memcpy(&v, p, 4); return v; }
    case kU32: { uint32_t v; memcpy(&v, p, 4); return v; }
    case kF32: { float v; memcpy(&v, p, 4); return v; }
    case kF64: { double v; memcpy(&v, p, 8); return v; }
    default: return 0.0;
    }
}

struct PlyProp {
    std::string name;
    PlyType type = kNone;        // scalar type, or the list's item type
    PlyType count_type = kNone;  // list count type (kNone: scalar property)
};

struct PlyElem {
    std::string name;
    long long count = 0;
    std::vector<PlyProp> props;
};

struct PlyHeader {
    int format = 0;  // 0 ascii, 1 binary_little_endian, 2 binary_big_endian
    std::vector<PlyElem> elems;
    long long nv = -1, nf = -1;
};

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v'; }

// One line of ASCII body: up to `max` numbers parsed with std::from_chars (the
// correctly rounded conversion strtof / strtol also perform).  Returns the
// count, or -1 on a malformed token.
template <class T>
int parse_line(const char* p, const char* e, T* out, int max) {
    int n = 0;
    for (;;) {
        while (p < e && is_space(*p)) p++;
        if (p >= e) return n;
        if (n == max) return max + 1;  // more tokens than the line may hold
        if (*p == '+') p++;
        const auto r = std::from_chars(p, e, out[n]);
        if (r.ec != std::errc() || (r.ptr < e && !is_space(*r.ptr))) return -1;
        p = r.ptr;
        n++;
    }
}

}  // namespace
}  // namespace rt

// Parallel ASCII body: one vertex (per_vertex numbers) and one face
// ("n i0 .. i(n-1)", n = 3 or 4) per line, which is what every PLY writer
// emits.  Files that do not keep to one record per line return false and take
// the token-by-token reader below (the reference's `>>` semantics).
static bool ply_ascii_lines(const char* p, const char* end, long long nv, long long nf, int per_vertex, int T,
                            std::vector<float>& verts, std::vector<int32_t>& arity, std::vector<int32_t>& idx) {
    std::vector<const char*> ls;  // starts of the first nv + nf non-blank lines
    ls.reserve((size_t)(nv + nf + 1));
    while (p < end && (long long)ls.size() < nv + nf) {
        const char* q = (const char*)memchr(p, '\n', (size_t)(end - p));
        const char* e = q ? q : end;
        const char* t = p;
        while (t < e && is_space(*t)) t++;
        if (t < e) ls.push_back(p);
        p = q ? q + 1 : end;
    }
    if ((long long)ls.size() < nv + nf) return false;
    auto line_end = [&](const char* s) {
        const char* q = (const char*)memchr(s, '\n', (size_t)(end - s));
        return q ? q : end;
    };
    verts.assign((size_t)nv * 3, 0.0f);
    arity.assign((size_t)nf, 0);
    std::vector<int32_t> quad((size_t)nf * 4, 0);
    std::atomic<bool> ok{true};
    const int64_t chunk = 8192;
    const int64_t nvc = (nv + chunk - 1) / chunk, nfc = (nf + chunk - 1) / chunk;
    parallel_for(nvc + nfc, T, [&](int64_t c) {
        if (c < nvc) {
            for (int64_t i = c * chunk; i < std::min<int64_t>(nv, (c + 1) * chunk) && ok; i++) {
                float v[8];
                const char* s = ls[(size_t)i];
                if (parse_line(s, line_end(s), v, per_vertex) != per_vertex) { ok = false; break; }
                for (int j = 0; j < 3; j++) verts[(size_t)i * 3 + j] = v[j];
            }
        } else {
            for (int64_t f = (c - nvc) * chunk; f < std::min<int64_t>(nf, (c - nvc + 1) * chunk) && ok; f++) {
                long v[6];
                const char* s = ls[(size_t)(nv + f)];
                const int n = parse_line(s, line_end(s), v, 5);
                if (n < 1 || (v[0] != 3 && v[0] != 4) || n != 1 + v[0]) { ok = false; break; }
                arity[(size_t)f] = (int32_t)v[0];
                for (int j = 0; j < v[0]; j++) quad[(size_t)f * 4 + j] = (int32_t)v[1 + j];
            }
        }
    });
    if (!ok) return false;
    idx.clear();
    idx.reserve((size_t)nf * 3);
    for (int64_t f = 0; f < nf; f++)
        for (int j = 0; j < arity[(size_t)f]; j++) idx.push_back(quad[(size_t)f * 4 + j]);
    return true;
}

// binary_little_endian body (the reference recognises the format,
// TD/read_ply.cpp:28, but reads no binary data): x, y, z of the vertex
// element (any scalar type, converted to float) and the face element's
// vertex-index list; other elements and properties are skipped by size.
static int ply_binary(const char* path, const rt::PlyHeader& H, const unsigned char* p, const unsigned char* end,
                      std::vector<float>& verts, std::vector<int32_t>& arity, std::vector<int32_t>& idx) {
    using namespace rt;
    for (const PlyElem& el : H.elems) {
        const bool is_v = el.name == "vertex", is_f = el.name == "face";
        int xyz[3] = {-1, -1, -1}, list = -1;
        for (size_t k = 0; k < el.props.size(); k++) {
            const PlyProp& pr = el.props[k];
            if (is_v && pr.count_type == kNone) {
                if (pr.name == "x") xyz[0] = (int)k;
                if (pr.name == "y") xyz[1] = (int)k;
                if (pr.name == "z") xyz[2] = (int)k;
            }
            if (is_f && pr.count_type != kNone && (list < 0 || pr.name == "vertex_indices" || pr.name == "vertex_index"))
                list = (int)k;
        }
        if (is_v) {
            if (xyz[0] < 0 || xyz[1] < 0 || xyz[2] < 0) return fail(RT_ERR_IO, "rt_read_ply: vertex x/y/z missing in %s", path);
            verts.assign((size_t)el.count * 3, 0.0f);
        }
        if (is_f) {
            if (list < 0) return fail(RT_ERR_IO, "rt_read_ply: face list missing in %s", path);
            arity.assign((size_t)el.count, 0);
            idx.reserve((size_t)el.count * 3);
        }
        for (long long i = 0; i < el.count; i++) {
            for (size_t k = 0; k < el.props.size(); k++) {
                const PlyProp& pr = el.props[k];
                if (pr.count_type == kNone) {
                    const int sz = ply_size(pr.type);
                    if (p + sz > end) return fail(RT_ERR_IO, "rt_read_ply: truncated %s", path);
                    if (is_v)
                        for (int j = 0; j < 3; j++)
                            if ((int)k == xyz[j]) verts[(size_t)i * 3 + j] = (float)ply_get(p, pr.type);
                    p += sz;
                } else {
                    const int csz = ply_size(pr.count_type), isz = ply_size(pr.type);
                    if (p + csz > end) return fail(RT_ERR_IO, "rt_read_ply: truncated %s", path);
                    const double cnt = ply_get(p, pr.count_type);
                    p += csz;
                    if (!(cnt >= 0) || p + (size_t)cnt * isz > end) return fail(RT_ERR_IO, "rt_read_ply: truncated %s", path);
                    if (is_f && (int)k == list) {
                        if (cnt != 3 && cnt != 4) return fail(RT_ERR_IO, "rt_read_ply: face %lld has %g vertices in %s", i, cnt, path);
                        arity[(size_t)i] = (int32_t)cnt;
                        for (int j = 0; j < (int)cnt; j++) idx.push_back((int32_t)ply_get(p + (size_t)j * isz, pr.type));
                    }
                    p += (size_t)cnt * isz;
                }
            }
        }
    }
    return RT_OK;
}

extern "C" int rt_read_ply(const char* path, int mode, float** points9, uint32_t* ntri,
                           rt_leaf_aabb** leafs) {
    if (!path) return fail(RT_ERR_INVALID, "rt_read_ply: null path");
    const int per_vertex = mode == 0 ? 3 : mode == 1 ? 5 : mode == 2 ? 6 : -1;
    if (per_vertex < 0) return fail(RT_ERR_INVALID, "rt_read_ply: unsupported mode %d", mode);
    FILE* fp = fopen(path, "rb");
    if (!fp) return fail(RT_ERR_IO, "rt_read_ply: cannot open %s", path);
    std::vector<char> buf;
    fseek(fp, 0, SEEK_END);
    long len = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    buf.resize((size_t)len + 1);
    size_t got = fread(buf.data(), 1, (size_t)len, fp);
    fclose(fp);
    buf[got] = 0;
    Cursor cur{buf.data(), buf.data() + got};
    std::string line;
    PlyHeader H;
    cur.line(line);
    if (line == "ply") cur.line(line);
    if (is_count_line(line)) {  // headerless prelude (H9 extension)
        H.nv = atoll(line.c_str());
        if (!cur.line(line) || !is_count_line(line)) return fail(RT_ERR_IO, "rt_read_ply: bad prelude in %s", path);
        H.nf = atoll(line.c_str());
    } else {                    // header loop, TD/read_ply.cpp:19-44
        for (;;) {
            char tag[64] = {0}, a1[64] = {0}, a2[64] = {0}, a3[64] = {0}, a4[64] = {0};
            const int nt = sscanf(line.c_str(), "%63s %63s %63s %63s %63s", tag, a1, a2, a3, a4);
            if (nt >= 2 && !strcmp(tag, "format")) {
                if (!strcmp(a1, "binary_little_endian")) H.format = 1;
                else if (!strcmp(a1, "binary_big_endian")) H.format = 2;
            } else if (nt >= 3 && !strcmp(tag, "element")) {
                PlyElem el;
                el.name = a1;
                el.count = atoll(a2);
                H.elems.push_back(el);
                if (el.name == "vertex") H.nv = el.count;
                if (el.name == "face") H.nf = el.count;
            } else if (nt >= 3 && !strcmp(tag, "property") && !H.elems.empty()) {
                PlyProp pr;
                if (!strcmp(a1, "list") && nt >= 5) {
                    pr.count_type = ply_type(a2);
                    pr.type = pr.count_type == kNone ? kNone : ply_type(a3);  // unknown types fail binary files
                    pr.name = a4;
                } else {
                    pr.type = ply_type(a1);
                    pr.name = a2;
                }
                H.elems.back().props.push_back(pr);
            }
            if (line == "end_header") break;
            if (!cur.line(line)) return fail(RT_ERR_IO, "rt_read_ply: no end_header in %s", path);
        }
    }
    if (H.nv < 0 || H.nf < 0) return fail(RT_ERR_IO, "rt_read_ply: missing vertex/face counts in %s", path);
    std::vector<float> verts;
    std::vector<int32_t> arity, idx;
    if (H.format == 2) return fail(RT_ERR_IO, "rt_read_ply: binary_big_endian is not supported (%s)", path);
    if (H.format == 1) {
        for (const PlyElem& el : H.elems)
            for (const PlyProp& pr : el.props)
                if (pr.type == kNone)
                    return fail(RT_ERR_IO, "rt_read_ply: unknown property type in %s", path);
        int rc = ply_binary(path, H, (const unsigned char*)cur.p, (const unsigned char*)cur.end, verts, arity, idx);
        if (rc) return rc;
        return rt_mesh_assemble(verts.data(), H.nv, arity.data(), idx.data(), H.nf, points9, ntri, leafs);
    }
    const long long nv = H.nv, nf = H.nf;
    if (!ply_ascii_lines(cur.p, cur.end, nv, nf, per_vertex, resolve_threads(0), verts, arity, idx)) {
        // token-by-token reader: the reference's sequential `>>` semantics
        verts.assign((size_t)nv * 3, 0.0f);
        const char* p = cur.p;
        for (long long i = 0; i < nv; i++)
            for (int j = 0; j < per_vertex; j++) {
                char* e;
                float v = strtof(p, &e);
                if (e == p) return fail(RT_ERR_IO, "rt_read_ply: bad vertex %lld in %s", i, path);
                p = e;
                if (j < 3) verts[(size_t)i * 3 + j] = v;
            }
        arity.assign((size_t)nf, 0);
        idx.clear();
        idx.reserve((size_t)nf * 3);
        for (long long f = 0; f < nf; f++) {
            char* e;
            long c = strtol(p, &e, 10);
            if (e == p || (c != 3 && c != 4)) return fail(RT_ERR_IO, "rt_read_ply: bad face %lld in %s", f, path);
            p = e;
            arity[(size_t)f] = (int32_t)c;
            for (long j = 0; j < c; j++) {
                long v = strtol(p, &e, 10);
                if (e == p) return fail(RT_ERR_IO, "rt_read_ply: bad face %lld in %s", f, path);
                p = e;
                idx.push_back((int32_t)v);
            }
        }
    }
    return rt_mesh_assemble(verts.data(), nv, arity.data(), idx.data(), nf, points9, ntri, leafs);
}

// ---------------------------------------------------------------- KD build

namespace {

// Lists in cut-flag order (TD/Trixel.h:172-193): 0 x1, 1 y1, 2 z1, 3 x0, 4 y0, 5 z0.
inline float list_key(const rt_leaf_aabb& a, int k) {
    switch (k) {
    case 0: return a.x1;
    case 1: return a.y1;
    case 2: return a.z1;
    case 3: return a.x0;
    case 4: return a.y0;
    default: return a.z0;
    }
}

struct Range { int64_t l, m, r; };

}  // namespace

namespace rt {
int validate_leafs(const rt_leaf_aabb* leafs, uint32_t n, const char* what) {
    if (!leafs || n == 0) return fail(RT_ERR_INVALID, "%s: empty input", what);
    if (n >= kLeafBit) return fail(RT_ERR_INVALID, "%s: too many triangles", what);
    // tri_list_index must be a permutation (set_sorted_voxels indexes by it)
    std::vector<uint8_t> seen(n, 0);
    for (uint32_t i = 0; i < n; i++) {
        int64_t t = leafs[i].tri;
        if (t < 0 || t >= (int64_t)n || seen[(size_t)t]) return fail(RT_ERR_INVALID, "%s: tri indices are not a permutation", what);
        seen[(size_t)t] = 1;
        for (int k = 0; k < 6; k++)
            if (isnan(list_key(leafs[i], k))) return fail(RT_ERR_INVALID, "%s: NaN bound at %u", what, i);
    }
    return RT_OK;
}
}  // namespace rt

namespace {

// A fixed pool of worker threads for the builder's many short parallel
// phases (about 100 per build): run(n, body) runs body(i) for i in [0, n)
// on the workers and the caller, and returns when all are done.  Spawning
// threads per phase (round 2) cost more than the phases on a many-core box.
class Pool {
public:
    explicit Pool(int threads) {
        for (int k = 1; k < threads; k++) workers_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    template <class F>
    void run(int64_t n, F&& body) {
        if (n <= 0) return;
        if (workers_.empty() || n == 1) {
            for (int64_t i = 0; i < n; i++) body(i);
            return;
        }
        std::function<void(int64_t)> f(body);
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &f;
            n_ = n;
            next_.store(0);
            busy_ = (int)workers_.size();
            gen_++;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [&] { return busy_ == 0; });
        fn_ = nullptr;
    }
    int size() const { return (int)workers_.size() + 1; }

private:
    void drain() {
        for (int64_t i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            drain();
            std::lock_guard<std::mutex> g(m_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::function<void(int64_t)>* fn_ = nullptr;
    int64_t n_ = 0;
    std::atomic<int64_t> next_{0};
    int busy_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Order-preserving unsigned image of a (non-NaN) float key, with -0.0 as
// +0.0: merge_sort compares with `<`, under which they are equal.
inline uint32_t key_bits(float f) {
    if (f == 0.0f) f = 0.0f;
    uint32_t u;
    memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int64_t kChunk = 1 << 15;  // elements per partition task

}  // namespace

extern "C" int rt_kd_build(const rt_leaf_aabb* leafs, uint32_t n, rt_kd_node* nodes, int nthreads) {
    if (!nodes) return fail(RT_ERR_INVALID, "rt_kd_build: null nodes");
    int vrc = validate_leafs(leafs, n, "rt_kd_build");
    if (vrc) return vrc;
    Pool pool(resolve_threads(nthreads));
    // Six sorted position lists.  merge_sort (TD/sort.h:25-60) takes the right
    // run on ties, so equal keys end up in descending input position: a
    // stable LSD radix sort (11 + 11 + 10 bits) of the order-preserving key
    // images, fed in descending position order, one list per task.
    std::vector<uint32_t> list[6], other[6];
    pool.run(6, [&](int64_t k) {
        std::vector<uint32_t> ka(n), kb(n), pb(n);
        auto& pa = list[k];
        pa.resize(n);
        other[k].resize(n);
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t pos = n - 1 - i;
            ka[i] = key_bits(list_key(leafs[pos], (int)k));
            pa[i] = pos;
        }
        uint32_t *K = ka.data(), *P = pa.data(), *K2 = kb.data(), *P2 = pb.data();
        static const int shift[3] = {0, 11, 22};
        for (int pass = 0; pass < 3; pass++) {
            uint32_t cnt[2049] = {0};
            const int sh = shift[pass];
            for (uint32_t i = 0; i < n; i++) cnt[((K[i] >> sh) & 2047u) + 1]++;
            for (int d = 0; d < 2048; d++) cnt[d + 1] += cnt[d];
            for (uint32_t i = 0; i < n; i++) {
                const uint32_t o = cnt[(K[i] >> sh) & 2047u]++;
                K2[o] = K[i];
                P2[o] = P[i];
            }
            std::swap(K, K2);
            std::swap(P, P2);
        }
        if (P != pa.data()) memcpy(pa.data(), P, sizeof(uint32_t) * n);  // odd pass count: result in pb
    });
    const int64_t nnode = 2 * (int64_t)n - 1;
    std::vector<Range> rng((size_t)nnode);
    std::vector<uint8_t> in_left(n, 0);
    pool.run((nnode + 65535) / 65536, [&](int64_t b) {  // (first touch of the caller's pages, in parallel)
        const int64_t a = b * 65536, e = std::min(nnode, a + 65536);
        memset(nodes + a, 0, sizeof(rt_kd_node) * (size_t)(e - a));
    });

    auto key_at = [&](int k, int64_t pos) { return list_key(leafs[list[k][(size_t)pos]], k); };

    rt_kd_node& root = nodes[0];
    root.parent = 0;
    root.cut_flag = 5;
    root.tri_index = -1;
    root.z1 = key_at(2, n - 1); root.z0 = key_at(5, 0);
    root.y1 = key_at(1, n - 1); root.y0 = key_at(4, 0);
    root.x0 = key_at(3, 0);     root.x1 = key_at(0, n - 1);
    rng[0] = {0, (int64_t)(n - 1) / 2, (int64_t)n - 1};

    // BFS one level at a time (TD/Trixel.h:135-385): nodes [lv0, lv1) are the
    // level's nodes, their ranges disjoint.  Each level: pick every node's
    // cut (strict `>`, H11) and finish its leaves; mark which elements go
    // left; stable-partition the five other lists of every interior node
    // (TD/Trixel.h:214-327) in chunks -- count each chunk's left elements,
    // scan within the node, scatter -- into the second buffer of each list
    // (the cut list is copied: its [l, m] is already the left child's); swap
    // the buffers; write the children (:329-376).
    struct Task { int64_t node, p0, p1; };
    std::vector<Task> tasks;
    std::vector<int64_t> child_base, task0, blocks;
    std::vector<uint32_t> lefts;  // [task][6]
    int64_t lv0 = 0, lv1 = 1, wr = 1;
    while (lv0 < lv1) {
        const int64_t cnt = lv1 - lv0;
        child_base.assign((size_t)cnt, -1);
        for (int64_t i = 0; i < cnt; i++) {
            const Range& R = rng[(size_t)(lv0 + i)];
            if (R.r != R.l) { child_base[(size_t)i] = wr; wr += 2; }
        }
        if (wr > nnode) return fail(RT_ERR_INVALID, "rt_kd_build: node overflow");
        // cut selection and leaves
        pool.run((cnt + 4095) / 4096, [&](int64_t blk) {
            for (int64_t i = blk * 4096; i < std::min(cnt, (blk + 1) * 4096); i++) {
                const int64_t id = lv0 + i;
                rt_kd_node& nd = nodes[id];
                const Range R = rng[(size_t)id];
                float best = key_at(0, R.r) - key_at(0, R.l);
                int cut = 0;
                static const int order[5] = {3, 1, 4, 2, 5};
                for (int q = 0; q < 5; q++) {
                    const int k = order[q];
                    float span = key_at(k, R.r) - key_at(k, R.l);
                    if (span > best) { best = span; cut = k; }
                }
                if (R.r == R.l) {  // leaf: TD/Trixel.h:194-205
                    nd.cut_flag = nodes[nd.parent].cut_flag;
                    nd.is_leaf = 1;
                    nd.left = -1; nd.right = -1;
                    nd.tri_index = leafs[list[0][(size_t)R.l]].tri;
                } else {
                    nd.cut_flag = cut;
                    nd.is_leaf = 0;
                    nd.tri_index = -1;
                }
            }
        });
        // the level's interior nodes in chunks of <= kChunk elements
        tasks.clear();
        task0.assign((size_t)cnt + 1, 0);
        for (int64_t i = 0; i < cnt; i++) {
            task0[(size_t)i] = (int64_t)tasks.size();
            const Range& R = rng[(size_t)(lv0 + i)];
            if (R.r == R.l) continue;
            for (int64_t p = R.l; p <= R.r; p += kChunk) tasks.push_back({i, p, std::min(R.r + 1, p + kChunk)});
        }
        task0[(size_t)cnt] = (int64_t)tasks.size();
        const int64_t nt = (int64_t)tasks.size();
        if (nt == 0) break;
        // runs of consecutive tasks of ~kChunk elements, one pool item each
        // (deep levels have a task per node: an item per task would make the
        // pool's work counter the bottleneck)
        blocks.clear();
        for (int64_t t = 0, acc = 0; t < nt; t++) {
            if (acc == 0) blocks.push_back(t);
            acc += tasks[(size_t)t].p1 - tasks[(size_t)t].p0;
            if (acc >= kChunk) acc = 0;
        }
        blocks.push_back(nt);
        const int64_t nb = (int64_t)blocks.size() - 1;
        // which elements go left: positions l..m of the node's cut list
        pool.run(nb, [&](int64_t j) {
            for (int64_t t = blocks[(size_t)j]; t < blocks[(size_t)j + 1]; t++) {
                const Task T = tasks[(size_t)t];
                const Range& R = rng[(size_t)(lv0 + T.node)];
                const auto& C = list[nodes[lv0 + T.node].cut_flag];
                for (int64_t p = T.p0; p < T.p1; p++) in_left[C[(size_t)p]] = p <= R.m ? 1 : 0;
            }
        });
        // left elements per chunk of the big nodes (a node of one chunk needs none)
        lefts.assign((size_t)nt * 6, 0);
        pool.run(nb * 6, [&](int64_t q) {
            const int k = (int)(q % 6);
            const uint32_t* L = list[k].data();
            for (int64_t t = blocks[(size_t)(q / 6)]; t < blocks[(size_t)(q / 6) + 1]; t++) {
                const Task T = tasks[(size_t)t];
                if (task0[(size_t)T.node + 1] - task0[(size_t)T.node] < 2 || k == (int)nodes[lv0 + T.node].cut_flag)
                    continue;
                uint32_t c = 0;
                for (int64_t p = T.p0; p < T.p1; p++) c += in_left[L[p]];
                lefts[(size_t)t * 6 + k] = c;
            }
        });
        // scatter: left elements from l + (lefts of earlier chunks), right
        // ones from m + 1 + (rights of earlier chunks)
        pool.run(nb * 6, [&](int64_t q) {
            const int k = (int)(q % 6);
            const uint32_t* L = list[k].data();
            uint32_t* O = other[k].data();
            for (int64_t t = blocks[(size_t)(q / 6)]; t < blocks[(size_t)(q / 6) + 1]; t++) {
                const Task T = tasks[(size_t)t];
                const Range& R = rng[(size_t)(lv0 + T.node)];
                if (k == (int)nodes[lv0 + T.node].cut_flag) {
                    memcpy(O + T.p0, L + T.p0, sizeof(uint32_t) * (size_t)(T.p1 - T.p0));
                    continue;
                }
                int64_t a = R.l, b = R.m + 1;
                for (int64_t u = task0[(size_t)T.node]; u < t; u++) {
                    const uint32_t c = lefts[(size_t)u * 6 + k];
                    a += c;
                    b += (tasks[(size_t)u].p1 - tasks[(size_t)u].p0) - c;
                }
                for (int64_t p = T.p0; p < T.p1; p++) {
                    const uint32_t e = L[p];
                    O[in_left[e] ? a++ : b++] = e;
                }
            }
        });
        for (int k = 0; k < 6; k++) list[k].swap(other[k]);
        // children (TD/Trixel.h:329-352), s1 / s2 (:353-376)
        pool.run((cnt + 4095) / 4096, [&](int64_t blk) {
            for (int64_t i = blk * 4096; i < std::min(cnt, (blk + 1) * 4096); i++) {
                const int64_t id = lv0 + i;
                const Range R = rng[(size_t)id];
                if (R.r == R.l) continue;
                rt_kd_node& nd = nodes[id];
                const int64_t cb = child_base[(size_t)i];
                nd.left = cb; nd.right = cb + 1;
                for (int br = 0; br < 2; br++) {
                    rt_kd_node& c = nodes[cb + br];
                    c.parent = id;
                    c.is_leaf = 0;
                    c.tri_index = -1;
                    int64_t nl = br == 0 ? R.l : R.m + 1, nr = br == 0 ? R.m : R.r;
                    rng[(size_t)(cb + br)] = {nl, ((nr - nl) / 2) + nl, nr};
                    c.x1 = key_at(0, nr); c.x0 = key_at(3, nl);
                    c.y1 = key_at(1, nr); c.y0 = key_at(4, nl);
                    c.z1 = key_at(2, nr); c.z0 = key_at(5, nl);
                }
                const rt_kd_node& Lc = nodes[cb];
                const rt_kd_node& Rc = nodes[cb + 1];
                switch (nd.cut_flag) {
                case 0: case 3: nd.s2 = Rc.x0; nd.s1 = Lc.x1; break;
                case 1: case 4: nd.s2 = Rc.y0; nd.s1 = Lc.y1; break;
                default:        nd.s2 = Rc.z0; nd.s1 = Lc.z1; break;
                }
            }
        });
        lv0 = lv1;
        lv1 = wr;
    }
    if (wr != nnode) return fail(RT_ERR_INVALID, "rt_kd_build: built %lld of %lld nodes", (long long)wr, (long long)nnode);
    return RT_OK;
}

// ------------------------------------------------------------------ camera

namespace {

// vector_norm, TD/vector.cpp:13-26 (8 Newton steps seeded from bits(s/2))
float host_vector_norm(float s) {
    const float half = 0.5f * s;
    union { float f; uint32_t i; } u;
    u.f = half;
    u.i = 0x5f375a86u - (u.i >> 1);
    for (int k = 0; k < 8; k++) u.f = u.f * (1.5f - half * u.f * u.f);
    return u.f;
}

struct V4 {
    float x, y, z, w;
    void normalize() {  // normalize_Vector(VEC4*), TD/Vector.h:116-124
        float s = x * x + y * y + z * z;
        s = host_vector_norm(s);
        x *= s; y *= s; z *= s;
        w = 1 / s;
    }
    void cross(const V4& b) {  // VEC4::cross, TD/vector.cpp:31-36
        float t0 = y * b.z - z * b.y;
        float t1 = z * b.x - x * b.z;
        float t2 = x * b.y - y * b.x;
        x = t0; y = t1; z = t2;
    }
};

}  // namespace

extern "C" float rt_film_w(int32_t w, int32_t h) {
    float ar = (float)w / (float)(uint32_t)h;  // TD/WinMain.cpp:29
    return ar * 0.024f;                        // TD/WinMain.cpp:70
}

extern "C" int rt_camera_basis(int32_t w, int32_t h, float f_w, float f_h, float focal,
                               const float pos[3], const float la[3], const float up[3],
                               rt_camera_basis_t* out) {
    if (!pos || !la || !up || !out || w <= 0 || h <= 0)
        return fail(RT_ERR_INVALID, "rt_camera_basis: bad argument");
    out->pix_w = f_w / (float)w;
    out->pix_h = f_h / (float)h;
    V4 n{la[0] - pos[0], la[1] - pos[1], la[2] - pos[2], 1.0f};
    n.normalize();
    out->n[0] = n.x; out->n[1] = n.y; out->n[2] = n.z;
    V4 tu{up[0], up[1], up[2], 1.0f};
    tu.normalize();
    tu.cross(n);          // up x n
    n.cross(tu);          // n x (up x n)
    V4 v = n;
    v.normalize();
    out->v[0] = v.x; out->v[1] = v.y; out->v[2] = v.z;
    for (int k = 0; k < 3; k++) out->v_mod[k] = out->v[k] * out->pix_h;
    V4 nn{la[0] - pos[0], la[1] - pos[1], la[2] - pos[2], 1.0f};
    nn.normalize();
    v.cross(nn);          // u = v x n
    out->u[0] = v.x; out->u[1] = v.y; out->u[2] = v.z;
    for (int k = 0; k < 3; k++) out->u_mod[k] = out->u[k] * out->pix_w;
    float adj_y = (float)((uint32_t)h >> 1);
    float adj_x = (float)((uint32_t)w >> 1);
    if (!((uint32_t)h & 1u)) adj_y = (float)((double)adj_y - .5);  // TD/Camera.cpp:62
    if (!((uint32_t)w & 1u)) adj_x = (float)((double)adj_x - .5);  // TD/Camera.cpp:63
    for (int k = 0; k < 3; k++)
        out->n_mod[k] = (out->n[k] * focal) - (out->v_mod[k] * adj_y) - (out->u_mod[k] * adj_x);
    return RT_OK;
}

extern "C" const char* rt_last_error_string(void) { return g_last_error.c_str(); }
extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }
