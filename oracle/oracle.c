/*
 * oracle/oracle.c -- CPU restatement of the reference ray-cast hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the parity checker and the timed
 * CPU baseline ("kind": "port").  Never linked into the product library.
 *
 * Built with -O3 -ffp-contract=off on x86-64 (SSE scalar float, no x87), so
 * every float expression below is evaluated in IEEE single precision in the
 * written order, and every expression the reference promotes to double
 * (1e-16 epsilons, `.6*`, `*.3`, `1.0/f`) is evaluated in double (SURVEY.md
 * §5 hazards H3/H4).  `powf(x,5)` (H5) is the shared deterministic pow5 used
 * by the HIP kernels as well.
 *
 * Reference paths: TD/ = TEST_Dungeonrun/.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_EPS 1e-16 /* MOLLER_TRUMBORE_DEVICE_EPSILON / DEVICE_EPSILON_SINGLE, TD/vector.cuh:10-11 */
#define ORC_DRAW_DISTANCE 400.0f        /* TD/Trixel.cu:47,176 */
#define ORC_BG 0x00F08200u              /* VEC4<T_uint>(240,130,0,0), TD/Camera.cpp:72 */
#define ORC_STACK_CAP 96

void orc_free(void* p) { free(p); }

/* ------------------------------------------------------------------ maths */

/* vector_norm, TD/vector.cpp:13-26.  Seed from the bits of s/2 (H7); the
 * union there is {float; s64}: the upper word is assumed zero (H6). */
float orc_host_vector_norm(float s) {
    float half = 0.5f * s;
    union { float f; uint32_t i; } u;
    u.f = half;
    u.i = 0x5f375a86u - (u.i >> 1);
    for (int k = 0; k < 8; k++) u.f = u.f * (1.5f - half * u.f * u.f);
    return u.f;
}

/* device_inverse_sqrt, TD/vector.cuh:79-95: one step then 20 more. */
float orc_device_inverse_sqrt(float x, float y, float z) {
    union { float f; uint32_t i; } u;
    u.f = (x * x) + (y * y) + (z * z);
    float half = 0.5f * u.f;
    u.f = half;
    u.i = 0x5f375a86u - (u.i >> 1);
    u.f = u.f * (1.5f - half * u.f * u.f);
    for (int k = 0; k < 20; k++) u.f = u.f * (1.5f - half * u.f * u.f);
    return u.f;
}

/* device_normalize_vector, TD/vector.cuh:116-120 */
static void dev_normalize(float* x, float* y, float* z) {
    float r = orc_device_inverse_sqrt(*x, *y, *z);
    *x *= r; *y *= r; *z *= r;
}

/* device_cross / device_dot, TD/vector.cuh:72-77,121-124 */
static void cross3(float* cx, float* cy, float* cz, float ax, float ay, float az,
                   float bx, float by, float bz) {
    *cx = ay * bz - az * by;
    *cy = az * bx - ax * bz;
    *cz = ax * by - ay * bx;
}
static float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return (ax * bx) + (ay * by) + (az * bz);
}

/* powf(|x|, 5) of TD/Camera.cu:45 (H5): evaluated in double, rounded once. */
static float pow5(float x) {
    double d = (double)x;
    double d2 = d * d;
    double d4 = d2 * d2;
    return (float)(d4 * d);
}

/* (u8)(float) of TD/Camera.cu:57-59 with NaN -> 0 (H14). */
static uint32_t to_u8(float t) {
    if (!(t >= 0.0f)) return 0u;
    if (t >= 256.0f) return 255u;
    return (uint32_t)(int)t;
}

/* -------------------------------------------------------------- PLY input */

/* min/max macros of windows.h as used in TD/read_ply.cpp:82-89,104-111,128-135 */
static float wmin(float a, float b) { return (a < b) ? a : b; }
static float wmax(float a, float b) { return (a > b) ? a : b; }

static void set_aabb(orc_leaf* lf, const float* a, const float* b, const float* c) {
    lf->x0 = wmin(a[0], wmin(b[0], c[0])); lf->x1 = wmax(a[0], wmax(b[0], c[0]));
    lf->y0 = wmin(a[1], wmin(b[1], c[1])); lf->y1 = wmax(a[1], wmax(b[1], c[1]));
    lf->z0 = wmin(a[2], wmin(b[2], c[2])); lf->z1 = wmax(a[2], wmax(b[2], c[2]));
    lf->sx0 = lf->sy0 = lf->sz0 = lf->sx1 = lf->sy1 = lf->sz1 = 0;
}

static void put3(float* dst, const float* v) { dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; }

/* Face assembly of TD/read_ply.cpp:67-149 (H8): a 4-gon ABCD becomes
 * (A,B,C),(A,C,D) with AABBs over {A,B,C} and {A,D,C}; a 3-gon P1P2P3 is
 * stored (P3,P1,P2) with its AABB over {P1,P2,P3}. */
int orc_assemble(const float* verts, int64_t nvert, const int32_t* arity,
                 const int32_t* idx, int64_t nface, float** points9,
                 uint32_t* ntri_out, orc_leaf** leafs_out) {
    int64_t ntri = 0;
    for (int64_t f = 0; f < nface; f++) {
        if (arity[f] == 3) ntri += 1;
        else if (arity[f] == 4) ntri += 2;
        else return -3;
    }
    float* pts = (float*)malloc(sizeof(float) * 9 * (size_t)(ntri ? ntri : 1));
    orc_leaf* lf = (orc_leaf*)calloc((size_t)(ntri ? ntri : 1), sizeof(orc_leaf));
    if (!pts || !lf) { free(pts); free(lf); return -2; }
    int64_t t = 0, k = 0;
    for (int64_t f = 0; f < nface; f++) {
        int a = arity[f];
        for (int j = 0; j < a; j++)
            if (idx[k + j] < 0 || idx[k + j] >= nvert) { free(pts); free(lf); return -4; }
        if (a == 4) {
            const float* A = verts + 3 * idx[k];
            const float* B = verts + 3 * idx[k + 1];
            const float* C = verts + 3 * idx[k + 2];
            const float* D = verts + 3 * idx[k + 3];
            set_aabb(&lf[t], A, B, C); lf[t].tri = t;
            put3(pts + 9 * t, A); put3(pts + 9 * t + 3, B); put3(pts + 9 * t + 6, C);
            t++;
            set_aabb(&lf[t], A, D, C); lf[t].tri = t;
            put3(pts + 9 * t, A); put3(pts + 9 * t + 3, C); put3(pts + 9 * t + 6, D);
            t++;
        } else {
            const float* P1 = verts + 3 * idx[k];
            const float* P2 = verts + 3 * idx[k + 1];
            const float* P3 = verts + 3 * idx[k + 2];
            set_aabb(&lf[t], P1, P2, P3); lf[t].tri = t;
            put3(pts + 9 * t, P3); put3(pts + 9 * t + 3, P1); put3(pts + 9 * t + 6, P2);
            t++;
        }
        k += a;
    }
    *points9 = pts;
    *leafs_out = lf;
    *ntri_out = (uint32_t)ntri;
    return 0;
}

static char* slurp(const char* path, size_t* len) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return NULL;
    fseek(fp, 0, SEEK_END);
    long n = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    char* buf = (char*)malloc((size_t)n + 1);
    if (!buf) { fclose(fp); return NULL; }
    size_t got = fread(buf, 1, (size_t)n, fp);
    fclose(fp);
    buf[got] = 0;
    *len = got;
    return buf;
}

/* Reads one line starting at *p (without the newline); advances *p. */
static size_t next_line(char** p, char* out, size_t cap) {
    size_t n = 0;
    while (**p && **p != '\n') {
        if (n + 1 < cap && **p != '\r') out[n++] = **p;
        (*p)++;
    }
    if (**p == '\n') (*p)++;
    out[n] = 0;
    return n;
}

static int is_uint_line(const char* s) {
    while (*s == ' ' || *s == '\t') s++;
    if (!(*s >= '0' && *s <= '9')) return 0;
    while (*s >= '0' && *s <= '9') s++;
    while (*s == ' ' || *s == '\t') s++;
    return *s == 0;
}

int orc_read_ply(const char* path, int mode, float** points9, uint32_t* ntri,
                 orc_leaf** leafs) {
    size_t len = 0;
    char* buf = slurp(path, &len);
    if (!buf) return -1;
    char* p = buf;
    char line[512];
    long nv = -1, nf = -1;
    next_line(&p, line, sizeof line);
    if (strcmp(line, "ply") == 0) next_line(&p, line, sizeof line);
    if (is_uint_line(line)) {
        /* headerless "nv\nnf\n" prelude (H9 extension) */
        nv = strtol(line, NULL, 10);
        next_line(&p, line, sizeof line);
        if (!is_uint_line(line)) { free(buf); return -5; }
        nf = strtol(line, NULL, 10);
    } else {
        /* header loop of TD/read_ply.cpp:19-44: spins until "end_header" */
        for (;;) {
            char tag[64] = {0}, name[64] = {0};
            long val = -1;
            int got = sscanf(line, "%63s %63s %ld", tag, name, &val);
            if (got >= 3 && strcmp(tag, "element") == 0) {
                if (strcmp(name, "vertex") == 0) nv = val;
                if (strcmp(name, "face") == 0) nf = val;
            }
            if (strcmp(line, "end_header") == 0) break;
            if (!*p) { free(buf); return -5; }
            next_line(&p, line, sizeof line);
        }
    }
    if (nv < 0 || nf < 0) { free(buf); return -5; }
    int per_vertex = mode == 0 ? 3 : mode == 1 ? 5 : mode == 2 ? 6 : -1;
    if (per_vertex < 0) { free(buf); return -6; }
    float* verts = (float*)malloc(sizeof(float) * 3 * (size_t)(nv ? nv : 1));
    int32_t* arity = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nf ? nf : 1));
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * 4 * (size_t)(nf ? nf : 1));
    if (!verts || !arity || !idx) { free(buf); free(verts); free(arity); free(idx); return -2; }
    for (long i = 0; i < nv; i++) {
        for (int j = 0; j < per_vertex; j++) {
            char* end;
            float v = strtof(p, &end);
            if (end == p) { free(buf); free(verts); free(arity); free(idx); return -7; }
            p = end;
            if (j < 3) verts[3 * i + j] = v;
        }
    }
    /* TD/read_ply.cpp:68: `for (i = 0; i < num_tri*3;)` with num_tri bumped
     * per quad reads exactly nf faces. */
    long k = 0;
    for (long f = 0; f < nf; f++) {
        char* end;
        long c = strtol(p, &end, 10);
        if (end == p || (c != 3 && c != 4)) { free(buf); free(verts); free(arity); free(idx); return -8; }
        p = end;
        arity[f] = (int32_t)c;
        for (long j = 0; j < c; j++) {
            long v = strtol(p, &end, 10);
            if (end == p) { free(buf); free(verts); free(arity); free(idx); return -8; }
            p = end;
            idx[k++] = (int32_t)v;
        }
    }
    free(buf);
    int rc = orc_assemble(verts, nv, arity, idx, nf, points9, ntri, leafs);
    free(verts); free(arity); free(idx);
    return rc;
}

/* -------------------------------------------------------------- KD build */

/* SORT_X0_TAG..SORT_Z1_TAG = 1..6, TD/sort.h:3-9 */
static float sort_key(const orc_leaf* a, int key) {
    switch (key) {
    case 1: return a->x0;
    case 2: return a->y0;
    case 3: return a->z0;
    case 4: return a->x1;
    case 5: return a->y1;
    default: return a->z1;
    }
}

/* _merge, TD/sort.h:25-60: a strict `<` takes the left element, so on ties
 * the right run goes first (H10). */
static void orc_merge(orc_leaf* a, uint32_t l, uint32_t m, uint32_t r, orc_leaf* w, int key) {
    uint32_t out = l, li = l, ri = m + 1;
    while (li <= m && ri <= r) {
        if (sort_key(&a[li], key) < sort_key(&a[ri], key)) w[out++] = a[li++];
        else w[out++] = a[ri++];
    }
    while (li <= m) w[out++] = a[li++];
    while (ri <= r) w[out++] = a[ri++];
    memcpy(a + l, w + l, sizeof(orc_leaf) * (size_t)(r - l + 1));
}

/* merge_recurse, TD/sort.h:16-23 */
static void orc_merge_rec(orc_leaf* a, uint32_t l, uint32_t r, orc_leaf* w, int key) {
    if (l >= r) return;
    uint32_t m = l + (r - l) / 2;
    orc_merge_rec(a, l, m, w, key);
    orc_merge_rec(a, m + 1, r, w, key);
    orc_merge(a, l, m, r, w, key);
}

void orc_merge_sort(orc_leaf* list, orc_leaf* work, uint32_t n, int key) {
    if (n == 0) return;
    orc_merge_rec(list, 0, n - 1, work, key);
}

/* The six lists in cut-flag order: 0 x1, 1 y1, 2 z1, 3 x0, 4 y0, 5 z0
 * (TD/Trixel.h:172-193,214-236).  Accessors for the list-k key and the
 * "position in list k" field. */
static float list_key(const orc_leaf* a, int k) {
    switch (k) {
    case 0: return a->x1;
    case 1: return a->y1;
    case 2: return a->z1;
    case 3: return a->x0;
    case 4: return a->y0;
    default: return a->z0;
    }
}
static int64_t* list_pos(orc_leaf* a, int k) {
    switch (k) {
    case 0: return &a->sx1;
    case 1: return &a->sy1;
    case 2: return &a->sz1;
    case 3: return &a->sx0;
    case 4: return &a->sy0;
    default: return &a->sz0;
    }
}

/* Trixel::set_sorted_voxels (TD/Trixel.h:386-473) then Trixel::create_kd
 * (TD/Trixel.h:135-385), restated with the same cross-index bookkeeping. */
int orc_build_kd(const orc_leaf* leafs, uint32_t n, orc_node* nodes) {
    if (n == 0) return -1;
    static const int tag_of_list[6] = {4, 5, 6, 1, 2, 3}; /* list k -> SORT tag */
    orc_leaf* lists[6];
    orc_leaf* work = (orc_leaf*)malloc(sizeof(orc_leaf) * n);
    orc_leaf* indexed = (orc_leaf*)malloc(sizeof(orc_leaf) * n);
    orc_leaf* tmp = (orc_leaf*)malloc(sizeof(orc_leaf) * (n + 20));
    if (!work || !indexed || !tmp) return -2;
    memcpy(indexed, leafs, sizeof(orc_leaf) * n);
    for (int k = 0; k < 6; k++) {
        lists[k] = (orc_leaf*)malloc(sizeof(orc_leaf) * n);
        memcpy(lists[k], leafs, sizeof(orc_leaf) * n);
        orc_merge_sort(lists[k], work, n, tag_of_list[k]);
    }
    /* indexed_leafs[tri].sorted_k_index = position of tri in list k (:427-434) */
    for (uint32_t i = 0; i < n; i++)
        for (int k = 0; k < 6; k++) {
            int64_t t = lists[k][i].tri;
            if (t < 0 || t >= (int64_t)n) return -3;
            *list_pos(&indexed[t], k) = i;
        }
    /* cross indices in every list (:436-466) */
    for (int k = 0; k < 6; k++)
        for (uint32_t i = 0; i < n; i++)
            for (int j = 0; j < 6; j++)
                *list_pos(&lists[k][i], j) = (j == k) ? (int64_t)i : *list_pos(&indexed[lists[k][i].tri], j);

    int64_t nnode = 2 * (int64_t)n - 1;
    memset(nodes, 0, sizeof(orc_node) * (size_t)nnode);
    for (int64_t i = 0; i < nnode; i++) { nodes[i].tri_index = -1; }
    int64_t rd = 0, wr = 1;
    orc_node* root = &nodes[0];
    root->l = 0; root->m = (n - 1) / 2; root->r = n - 1;
    root->parent = 0; root->cut_flag = 5; root->is_leaf = 0;
    root->z1 = lists[2][n - 1].z1; root->z0 = lists[5][0].z0;
    root->y1 = lists[1][n - 1].y1; root->y0 = lists[4][0].y0;
    root->x0 = lists[3][0].x0;     root->x1 = lists[0][n - 1].x1;

    while (rd < wr) {
        orc_node* cur = &nodes[rd];
        int64_t l = cur->l, m = cur->m, r = cur->r;
        /* axis/key selection, strict `>` in the order x1,x0,y1,y0,z1,z0 (H11) */
        float best = list_key(&lists[0][r], 0) - list_key(&lists[0][l], 0);
        int cut = 0;
        static const int order[5] = {3, 1, 4, 2, 5};
        for (int q = 0; q < 5; q++) {
            int k = order[q];
            float span = list_key(&lists[k][r], k) - list_key(&lists[k][l], k);
            if (span > best) { best = span; cut = k; }
        }
        cur->cut_flag = (r - l) != 0 ? cut : nodes[cur->parent].cut_flag;
        if (r == l) {
            cur->left = -1; cur->right = -1; cur->is_leaf = 1;
            cur->tri_index = lists[0][l].tri;
            rd++;
            continue;
        }
        /* stable partition of every non-cut list around the median (:214-327) */
        for (int li = 0; li < 6; li++) {
            if (li == cur->cut_flag) continue;
            orc_leaf* f = lists[li];
            int64_t lcount = 0, rcount = m - l + 1;
            for (int64_t i = l; i <= r; i++) {
                int64_t pivot = *list_pos(&f[i], cur->cut_flag);
                int64_t t = pivot <= m ? lcount++ : rcount++;
                for (int j = 0; j < 6; j++)
                    *list_pos(&tmp[t], j) = (j == li) ? l + t : *list_pos(&f[i], j);
                for (int s = 0; s < 6; s++) {
                    if (s == li) continue;
                    *list_pos(&lists[s][*list_pos(&tmp[t], s)], li) = l + t;
                }
                tmp[t].x0 = f[i].x0; tmp[t].x1 = f[i].x1;
                tmp[t].y0 = f[i].y0; tmp[t].y1 = f[i].y1;
                tmp[t].z0 = f[i].z0; tmp[t].z1 = f[i].z1;
                tmp[t].tri = f[i].tri;
            }
            memcpy(f + l, tmp, sizeof(orc_leaf) * (size_t)(r - l + 1));
        }
        /* children in BFS order, right = left + 1 (:329-352) */
        for (int branch = 0; branch < 2; branch++) {
            orc_node* c = &nodes[wr];
            c->parent = rd; c->is_leaf = 0;
            int64_t nl, nr;
            if (branch == 0) { nl = l; nr = m; cur->left = wr; }
            else { nl = m + 1; nr = r; cur->right = wr; }
            c->l = nl; c->r = nr; c->m = ((nr - nl) / 2) + nl;
            c->x1 = lists[0][nr].x1; c->x0 = lists[3][nl].x0;
            c->y1 = lists[1][nr].y1; c->y0 = lists[4][nl].y0;
            c->z1 = lists[2][nr].z1; c->z0 = lists[5][nl].z0;
            wr++;
        }
        /* s1 = left child's max, s2 = right child's min on the cut axis (:353-376) */
        orc_node* L = &nodes[wr - 2];
        orc_node* R = &nodes[wr - 1];
        switch (cur->cut_flag) {
        case 0: case 3: cur->s2 = R->x0; cur->s1 = L->x1; break;
        case 1: case 4: cur->s2 = R->y0; cur->s1 = L->y1; break;
        default:        cur->s2 = R->z0; cur->s1 = L->z1; break;
        }
        rd++;
    }
    for (int k = 0; k < 6; k++) free(lists[k]);
    free(work); free(indexed); free(tmp);
    return wr == nnode ? 0 : -4;
}

/* ---------------------------------------------------------------- camera */

static void host_normalize4(float v[4]) {
    /* normalize_Vector(VEC4*), TD/Vector.h:116-124 */
    float s = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    s = orc_host_vector_norm(s);
    v[0] *= s; v[1] *= s; v[2] *= s;
    v[3] = 1 / s;
}
static void host_cross4(float a[4], const float b[4]) {
    /* VEC4::cross, TD/vector.cpp:31-36 */
    float t0 = a[1] * b[2] - a[2] * b[1];
    float t1 = a[2] * b[0] - a[0] * b[2];
    float t2 = a[0] * b[1] - a[1] * b[0];
    a[0] = t0; a[1] = t1; a[2] = t2;
}

float orc_film_w(int32_t w, int32_t h) {
    float ar = (float)w / (float)(uint32_t)h; /* TD/WinMain.cpp:29 */
    return ar * 0.024f;                       /* TD/WinMain.cpp:70 */
}

void orc_camera_basis(int32_t w, int32_t h, float f_w, float f_h, float focal,
                      const float pos[3], const float la[3], const float up[3],
                      orc_camera* c) {
    memset(c, 0, sizeof *c);
    c->w = w; c->h = h;
    c->pix_w = f_w / (float)w;
    c->pix_h = f_h / (float)h;
    for (int k = 0; k < 3; k++) c->pos[k] = pos[k];
    float tn[4] = {la[0] - pos[0], la[1] - pos[1], la[2] - pos[2], 1.0f};
    host_normalize4(tn);
    for (int k = 0; k < 3; k++) c->n[k] = tn[k];
    float tu[4] = {up[0], up[1], up[2], 1.0f};
    host_normalize4(tu);
    host_cross4(tu, tn);
    host_cross4(tn, tu);
    float tv[4] = {tn[0], tn[1], tn[2], tn[3]};
    host_normalize4(tv);
    for (int k = 0; k < 3; k++) { c->v[k] = tv[k]; c->v_mod[k] = c->v[k] * c->pix_h; }
    float tuu[4] = {la[0] - pos[0], la[1] - pos[1], la[2] - pos[2], 1.0f};
    host_normalize4(tuu);
    host_cross4(tv, tuu);
    for (int k = 0; k < 3; k++) { c->u[k] = tv[k]; c->u_mod[k] = c->u[k] * c->pix_w; }
    float adj_y = (float)((uint32_t)h >> 1);
    float adj_x = (float)((uint32_t)w >> 1);
    if (!((uint32_t)h & 1u)) adj_y = (float)((double)adj_y - .5);
    if (!((uint32_t)w & 1u)) adj_x = (float)((double)adj_x - .5);
    for (int k = 0; k < 3; k++)
        c->n_mod[k] = (c->n[k] * focal) - (c->v_mod[k] * adj_y) - (c->u_mod[k] * adj_x);
}

void orc_primary_ray(const orc_camera* c, int32_t ix, int32_t iy, float out[3]) {
    /* init_cam_mem_cuda, TD/Camera.cu:103-104 */
    float fx = (float)(uint64_t)ix, fy = (float)(uint64_t)iy;
    float x = c->n_mod[0] + c->u_mod[0] * fx + c->v_mod[0] * fy;
    float y = c->n_mod[1] + c->u_mod[1] * fx + c->v_mod[1] * fy;
    float z = c->n_mod[2] + c->u_mod[2] * fx + c->v_mod[2] * fy;
    dev_normalize(&x, &y, &z);
    out[0] = x; out[1] = y; out[2] = z;
}

/* ----------------------------------------------------------------- scene */

struct orc_scene {
    uint32_t ntri;
    int64_t nnode;
    orc_camera cam;
    /* Trixel::trixel_memory (TD/Trixel.h:56-66) */
    float *p1, *e1, *e2, *nrm, *rad;   /* 3 floats per triangle, AoS */
    /* Camera::trixel_memory (TD/Camera.h:64-68) */
    float *dt, *dq, *dw;
    /* Camera::voxel_memory (TD/Camera.h:69-84) */
    float* bo;      /* t0x,t0y,t0z,t1x,t1y,t1z */
    float *s1, *s2;
    uint8_t* is_leaf;
    int64_t *left, *right, *tri;
    uint8_t* cut;   /* x,y,z one-hot */
    int32_t qoff;   /* index_queue_offset, TD/Camera.cpp:202-203 */
};

orc_scene* orc_scene_create(const float* pts, const float* rad3, uint32_t ntri,
                            const orc_node* nodes, const orc_camera* cam) {
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    s->ntri = ntri;
    s->nnode = nodes ? 2 * (int64_t)ntri - 1 : 0;
    s->cam = *cam;
    size_t n3 = sizeof(float) * 3 * (size_t)ntri;
    s->p1 = (float*)malloc(n3); s->e1 = (float*)malloc(n3); s->e2 = (float*)malloc(n3);
    s->nrm = (float*)malloc(n3); s->rad = (float*)malloc(n3);
    s->dt = (float*)malloc(n3); s->dq = (float*)malloc(n3);
    s->dw = (float*)malloc(sizeof(float) * (size_t)ntri);
    for (uint32_t i = 0; i < ntri; i++) {
        const float* P = pts + 9 * (size_t)i;
        /* init_tri_mem_cuda, TD/Trixel.cu:11-27 */
        float* p1 = s->p1 + 3 * i; float* e1 = s->e1 + 3 * i;
        float* e2 = s->e2 + 3 * i; float* n = s->nrm + 3 * i;
        p1[0] = P[0]; p1[1] = P[1]; p1[2] = P[2];
        e1[0] = P[3] - P[0]; e1[1] = P[4] - P[1]; e1[2] = P[5] - P[2];
        e2[0] = P[6] - P[0]; e2[1] = P[7] - P[1]; e2[2] = P[8] - P[2];
        cross3(&n[0], &n[1], &n[2], e1[0], e1[1], e1[2], e2[0], e2[1], e2[2]);
        dev_normalize(&n[0], &n[1], &n[2]);
        for (int k = 0; k < 3; k++) s->rad[3 * i + k] = rad3[3 * i + k];
        /* init_cam_tri_mem_cuda, TD/Trixel.cu:29-36 */
        float* dt = s->dt + 3 * i; float* dq = s->dq + 3 * i;
        dt[0] = cam->pos[0] - p1[0]; dt[1] = cam->pos[1] - p1[1]; dt[2] = cam->pos[2] - p1[2];
        cross3(&dq[0], &dq[1], &dq[2], dt[0], dt[1], dt[2], e1[0], e1[1], e1[2]);
        s->dw[i] = dot3(dq[0], dq[1], dq[2], e2[0], e2[1], e2[2]);
    }
    if (nodes) {
        int64_t nn = s->nnode;
        s->bo = (float*)malloc(sizeof(float) * 6 * (size_t)nn);
        s->s1 = (float*)malloc(sizeof(float) * (size_t)nn);
        s->s2 = (float*)malloc(sizeof(float) * (size_t)nn);
        s->is_leaf = (uint8_t*)malloc((size_t)nn);
        s->left = (int64_t*)malloc(sizeof(int64_t) * (size_t)nn);
        s->right = (int64_t*)malloc(sizeof(int64_t) * (size_t)nn);
        s->tri = (int64_t*)malloc(sizeof(int64_t) * (size_t)nn);
        s->cut = (uint8_t*)malloc(3 * (size_t)nn);
        const float co[3] = {cam->pos[0], cam->pos[1], cam->pos[2]};
        const float oc[3] = {0.0f, 0.0f, 0.0f}; /* obj_center, TD/Camera.cpp:167-170 */
        for (int64_t i = 0; i < nn; i++) {
            /* init_cam_voxel_mem_cuda, TD/Camera.cu:137-162 */
            const orc_node* nd = &nodes[i];
            int cd = nd->cut_flag;
            float* b = s->bo + 6 * i;
            b[0] = nd->x0 - co[0] + oc[0];
            b[3] = nd->x1 - co[0] + oc[0];
            b[1] = nd->y0 - co[1] + oc[1];
            b[4] = nd->y1 - co[1] + oc[1];
            b[2] = nd->z0 - co[2] + oc[2];
            b[5] = nd->z1 - co[2] + oc[2];
            s->is_leaf[i] = (uint8_t)nd->is_leaf;
            s->left[i] = nd->left; s->right[i] = nd->right;
            s->tri[i] = s->is_leaf[i] == 0 ? -1 : nd->tri_index;
            uint8_t cx = (cd == 0 || cd == 3), cy = (cd == 1 || cd == 4), cz = (cd == 2 || cd == 5);
            s->cut[3 * i] = cx; s->cut[3 * i + 1] = cy; s->cut[3 * i + 2] = cz;
            s->s1[i] = nd->s1 - (((co[0] + oc[0]) * (float)cx) + ((co[1] + oc[1]) * (float)cy) + ((co[2] + oc[2]) * (float)cz));
            /* the reference's obj_center.x typo on the z term is kept (it is 0) */
            s->s2[i] = nd->s2 - (((co[0] + oc[0]) * (float)cx) + ((co[1] + oc[1]) * (float)cy) + ((co[2] + oc[0]) * (float)cz));
        }
        s->qoff = (int32_t)ceil(log2((double)nn));
    }
    return s;
}

void orc_scene_destroy(orc_scene* s) {
    if (!s) return;
    free(s->p1); free(s->e1); free(s->e2); free(s->nrm); free(s->rad);
    free(s->dt); free(s->dq); free(s->dw);
    free(s->bo); free(s->s1); free(s->s2); free(s->is_leaf);
    free(s->left); free(s->right); free(s->tri); free(s->cut);
    free(s);
}

/* --------------------------------------------------------------- shading */

uint32_t orc_phong(const float pnt[3], const float nrm[3], const float rmd[3],
                   const float rad[3]) {
    /* color_cam_cuda, TD/Camera.cu:27-60 */
    float sdx = 2 - pnt[0], sdy = 2 - pnt[1], sdz = 2 - pnt[2];
    dev_normalize(&sdx, &sdy, &sdz);
    float dot_r_n = dot3(sdx, sdy, sdz, nrm[0], nrm[0], nrm[2]); /* H1: norm.x twice */
    float rx = (sdx - (2 * dot_r_n * nrm[0])) * rmd[0];
    float ry = (sdy - (2 * dot_r_n * nrm[1])) * rmd[1];
    float rz = (sdz - (2 * dot_r_n * nrm[2])) * rmd[2];
    float diff = (float)(.6 * (double)fabsf(dot_r_n));
    float spec = (float)((double)pow5(fabsf((rx + ry + rz))) * .3);
    float pr = 0.0f, pg = 0.0f, pb = 0.0f;
    pr += (rad[0] * diff) + (1 * spec);
    pg += (rad[1] * diff) + (1 * spec);
    pb += (rad[2] * diff) + (1 * spec);
    float mx = fmaxf(fmaxf(pr, pg), pb);
    uint32_t r8 = to_u8((pr / mx) * 255);
    uint32_t g8 = to_u8((pg / mx) * 255);
    uint32_t b8 = to_u8((pb / mx) * 255);
    return (r8 << 16) | (g8 << 8) | b8;
}

/* ------------------------------------------------------------- intersect */

typedef struct {
    int64_t rmi;
    float d;
    float rad[3], pnt[3], nrm[3];
    float r[3], od[3];   /* the object-space ray and translation used */
} orc_hit;

/* intersect_voxel_cuda, TD/Trixel.cu:41-172, one pixel. */
static int trace_kd(const orc_scene* s, const float* X, const float cam_rmd[3],
                    orc_hit* out, uint64_t* cnt) {
    float d = ORC_DRAW_DISTANCE;
    int32_t stack[ORC_STACK_CAP];
    int top = 0, rc = 0;
    stack[0] = 0;
    out->rmi = -1;
    float odx = X[3], ody = X[7], odz = X[11];
    float rx = -1 * (X[0] * -cam_rmd[0] + X[1] * -cam_rmd[1] + X[2] * -cam_rmd[2]);
    float ry = -1 * (X[4] * -cam_rmd[0] + X[5] * -cam_rmd[1] + X[6] * -cam_rmd[2]);
    float rz = -1 * (X[8] * -cam_rmd[0] + X[9] * -cam_rmd[1] + X[10] * -cam_rmd[2]);
    out->r[0] = rx; out->r[1] = ry; out->r[2] = rz;
    out->od[0] = odx; out->od[1] = ody; out->od[2] = odz;
    while (top >= 0) {
        int32_t cni = stack[top--];
        if (s->is_leaf[cni]) {
            cnt[ORC_CNT_LEAF]++;
            int64_t t = s->tri[cni];
            const float* e1 = s->e1 + 3 * t; const float* e2 = s->e2 + 3 * t;
            const float* dt = s->dt + 3 * t;
            float px, py, pz;
            cross3(&px, &py, &pz, rx, ry, rz, e2[0], e2[1], e2[2]);
            float f = dot3(px, py, pz, e1[0], e1[1], e1[2]);
            if (!((double)f < ORC_EPS && (double)f > -ORC_EPS)) {
                float pe1 = (float)(1.0 / (double)f);
                float tx = dt[0] - odx, ty = dt[1] - ody, tz = dt[2] - odz;
                float u = pe1 * dot3(px, py, pz, tx, ty, tz);
                float qx, qy, qz;
                cross3(&qx, &qy, &qz, tx, ty, tz, e1[0], e1[1], e1[2]);
                float v = pe1 * dot3(rx, ry, rz, qx, qy, qz);
                float w = pe1 * dot3(e2[0], e2[1], e2[2], qx, qy, qz);
                if ((w < d) && !(((double)u < ORC_EPS) || ((double)v < ORC_EPS) ||
                                 ((double)(u + v) > 1 + ORC_EPS) || ((double)w < ORC_EPS))) {
                    cnt[ORC_CNT_ACCEPT]++;
                    d = w;
                    out->rmi = t;
                    out->d = w;
                    for (int k = 0; k < 3; k++) out->rad[k] = s->rad[3 * t + k];
                    out->pnt[0] = d * rx + odx;
                    out->pnt[1] = d * ry + ody;
                    out->pnt[2] = d * rz + odz;
                    /* norm.device_rotate(rot_m, i, -1), TD/vector.cuh:23-33 */
                    const float* n = s->nrm + 3 * t;
                    float ax = -1 * n[0], ay = -1 * n[1], az = -1 * n[2];
                    float nx = ax * X[0] + ay * X[1] + az * X[2];
                    float ny = ax * X[4] + ay * X[5] + az * X[6];
                    float nz = ax * X[8] + ay * X[9] + az * X[10];
                    out->nrm[0] = nx * -1; out->nrm[1] = ny * -1; out->nrm[2] = nz * -1;
                }
            }
            continue;
        }
        cnt[ORC_CNT_INTERIOR]++;
        const float* b = s->bo + 6 * (int64_t)cni;
        float t0x = rx > 0 ? b[0] * (1 / rx) : b[3] * (1 / rx);
        float t1x = rx > 0 ? b[3] * (1 / rx) : b[0] * (1 / rx);
        float t0y = ry > 0 ? b[1] * (1 / ry) : b[4] * (1 / ry);
        float t1y = ry > 0 ? b[4] * (1 / ry) : b[1] * (1 / ry);
        float t0z = rz > 0 ? b[2] * (1 / rz) : b[5] * (1 / rz);
        float t1z = rz > 0 ? b[5] * (1 / rz) : b[2] * (1 / rz);
        const uint8_t* cf = s->cut + 3 * (int64_t)cni;
        float dir = ((rx * cf[0]) + (ry * cf[1]) + (rz * cf[2]));
        float ds = ((odx * cf[0]) + (ody * cf[1]) + (odz * cf[2]));
        float maxt0 = fmaxf(t0z + odz / rz, fmaxf(t0x + odx / rx, t0y + ody / ry));
        float mint1 = fminf(t1z + odz / rz, fminf(t1x + odx / rx, t1y + ody / ry));
        if ((double)mint1 >= (double)maxt0 - ORC_EPS && (double)maxt0 > -ORC_EPS) {
            cnt[ORC_CNT_DESCEND]++;
            maxt0 *= dir; mint1 *= dir;
            float s1 = (float)((double)s->s1[cni] + ORC_EPS + (double)ds);
            float s2 = s->s2[cni] + ds;
            int32_t L = (int32_t)s->left[cni], R = (int32_t)s->right[cni];
            if ((double)maxt0 < (double)s2 + ORC_EPS) {
                if ((double)mint1 > (double)s2 - ORC_EPS) stack[++top] = R;
                stack[++top] = L;
            } else {
                if (mint1 < s1 || maxt0 < s1) stack[++top] = L;
                stack[++top] = R;
            }
            if (top + 1 > (int)cnt[ORC_CNT_MAXSTACK]) cnt[ORC_CNT_MAXSTACK] = (uint64_t)(top + 1);
            if (top + 1 > s->qoff && s->qoff > 0) rc = -1;
            if (top + 2 >= ORC_STACK_CAP) return -1;
        }
    }
    return rc;
}

/* Shadow ray, one per hit.  Not in the
 * reference: its hook is the commented-out test at TD/Camera.cu:28-34, so
 * the definition is ours, shared bit for bit with the kernels:
 *   - the occluder test is the segment between the light (2,2,2) of
 *     TD/Camera.cu:32 and the primary hit H = d*r - od (the point the
 *     traversal's own origin -od reaches, TD/Trixel.cu:90-109; H == pnt
 *     for the identity transform);
 *   - the segment is walked FROM THE LIGHT: the reference's box-entry rule
 *     (maxt0 > -eps, TD/Trixel.cu:95) culls every box that contains the
 *     origin, so a ray leaving the surface would cull the root.  From the
 *     light (outside the model) the reference's rules apply unchanged:
 *     origin via the translation od_L = -(2,2,2), direction
 *     s = normalize(H - (2,2,2)) with the 21-step device rsqrt;
 *   - it is shadowed iff some visited leaf other than the hit triangle passes
 *     the MT tests (TD/Trixel.cu:104-120) with w < Lmax,
 *     Lmax = |H - (2,2,2)| * (1 - 2^-10) (a relative bias, exact in f32);
 *   - the walk is the segment's: a box is entered only where the segment
 *     enters it, i.e. the reference's entry test (TD/Trixel.cu:95) with its
 *     entry parameter also below Lmax (maxt0 < Lmax, the float maxt0 of the
 *     test).  Round 6: before it the walk followed the whole ray beyond H;
 *     every committed shadow frame is the same image with either walk
 *     (tests/golden/frame_hashes.json), and the segment's walk visits
 *     24-45 % fewer nodes;
 *   - a shadowed pixel keeps point_rad = 0, so the reference's formula gives
 *     0/0 -> (u8)NaN = 0 in every channel: 0x00000000 (H14).
 * Any-hit is an OR over the visited leaves, so the result does not depend on
 * the visiting order.  Every leaf is visited here (no early exit) so the visit
 * counters are deterministic; the kernels stop early unless counting. */
#define ORC_SHADOW_SCALE 0.9990234375f

static int trace_shadow(const orc_scene* s, const float r[3], const float od[3], float L, int64_t self,
                        uint64_t* cnt) {
    int32_t stack[ORC_STACK_CAP];
    int top = 0, shadowed = 0;
    stack[0] = 0;
    const float rx = r[0], ry = r[1], rz = r[2], odx = od[0], ody = od[1], odz = od[2];
    while (top >= 0) {
        int32_t cni = stack[top--];
        if (s->is_leaf[cni]) {
            cnt[ORC_CNT_LEAF]++;
            int64_t t = s->tri[cni];
            const float* e1 = s->e1 + 3 * t; const float* e2 = s->e2 + 3 * t;
            const float* dt = s->dt + 3 * t;
            float px, py, pz;
            cross3(&px, &py, &pz, rx, ry, rz, e2[0], e2[1], e2[2]);
            float f = dot3(px, py, pz, e1[0], e1[1], e1[2]);
            if (!((double)f < ORC_EPS && (double)f > -ORC_EPS)) {
                float pe1 = (float)(1.0 / (double)f);
                float tx = dt[0] - odx, ty = dt[1] - ody, tz = dt[2] - odz;
                float u = pe1 * dot3(px, py, pz, tx, ty, tz);
                float qx, qy, qz;
                cross3(&qx, &qy, &qz, tx, ty, tz, e1[0], e1[1], e1[2]);
                float v = pe1 * dot3(rx, ry, rz, qx, qy, qz);
                float w = pe1 * dot3(e2[0], e2[1], e2[2], qx, qy, qz);
                if ((w < L) && !(((double)u < ORC_EPS) || ((double)v < ORC_EPS) ||
                                 ((double)(u + v) > 1 + ORC_EPS) || ((double)w < ORC_EPS)) &&
                    t != self) {
                    cnt[ORC_CNT_ACCEPT]++;
                    shadowed = 1;
                }
            }
            continue;
        }
        cnt[ORC_CNT_INTERIOR]++;
        const float* b = s->bo + 6 * (int64_t)cni;
        float t0x = rx > 0 ? b[0] * (1 / rx) : b[3] * (1 / rx);
        float t1x = rx > 0 ? b[3] * (1 / rx) : b[0] * (1 / rx);
        float t0y = ry > 0 ? b[1] * (1 / ry) : b[4] * (1 / ry);
        float t1y = ry > 0 ? b[4] * (1 / ry) : b[1] * (1 / ry);
        float t0z = rz > 0 ? b[2] * (1 / rz) : b[5] * (1 / rz);
        float t1z = rz > 0 ? b[5] * (1 / rz) : b[2] * (1 / rz);
        const uint8_t* cf = s->cut + 3 * (int64_t)cni;
        float dir = ((rx * cf[0]) + (ry * cf[1]) + (rz * cf[2]));
        float ds = ((odx * cf[0]) + (ody * cf[1]) + (odz * cf[2]));
        float maxt0 = fmaxf(t0z + odz / rz, fmaxf(t0x + odx / rx, t0y + ody / ry));
        float mint1 = fminf(t1z + odz / rz, fminf(t1x + odx / rx, t1y + ody / ry));
        if ((double)mint1 >= (double)maxt0 - ORC_EPS && (double)maxt0 > -ORC_EPS && maxt0 < L) {
            cnt[ORC_CNT_DESCEND]++;
            maxt0 *= dir; mint1 *= dir;
            float s1 = (float)((double)s->s1[cni] + ORC_EPS + (double)ds);
            float s2 = s->s2[cni] + ds;
            int32_t Lc = (int32_t)s->left[cni], Rc = (int32_t)s->right[cni];
            if ((double)maxt0 < (double)s2 + ORC_EPS) {
                if ((double)mint1 > (double)s2 - ORC_EPS) stack[++top] = Rc;
                stack[++top] = Lc;
            } else {
                if (mint1 < s1 || maxt0 < s1) stack[++top] = Lc;
                stack[++top] = Rc;
            }
            if (top + 2 >= ORC_STACK_CAP) return -1;
        }
    }
    return shadowed;
}

/* The shadow ray of a primary hit (see trace_shadow): direction, translated
 * origin and segment length, exactly as the kernels compute them. */
static void shadow_ray(const orc_hit* h, float sdir[3], float od_l[3], float* Lmax) {
    float sx = ((h->d * h->r[0]) - h->od[0]) - 2;
    float sy = ((h->d * h->r[1]) - h->od[1]) - 2;
    float sz = ((h->d * h->r[2]) - h->od[2]) - 2;
    float L = (float)sqrt((double)((sx * sx) + (sy * sy) + (sz * sz)));
    *Lmax = L * ORC_SHADOW_SCALE;
    dev_normalize(&sx, &sy, &sz);
    sdir[0] = sx; sdir[1] = sy; sdir[2] = sz;
    od_l[0] = -2; od_l[1] = -2; od_l[2] = -2;
}

/* intersect_trixel_cuda, TD/Trixel.cu:173-209, one pixel (never launched by
 * the reference; BASELINE config 2). */
static void trace_flat(const orc_scene* s, const float rmd[3], orc_hit* out, uint64_t* cnt) {
    float d = ORC_DRAW_DISTANCE;
    out->rmi = -1;
    for (uint32_t t = 0; t < s->ntri; t++) {
        const float* e1 = s->e1 + 3 * (size_t)t; const float* e2 = s->e2 + 3 * (size_t)t;
        const float* dt = s->dt + 3 * (size_t)t; const float* dq = s->dq + 3 * (size_t)t;
        float px, py, pz;
        cross3(&px, &py, &pz, rmd[0], rmd[1], rmd[2], e2[0], e2[1], e2[2]);
        float f = dot3(px, py, pz, e1[0], e1[1], e1[2]);
        if (!((double)f < ORC_EPS && (double)f > -ORC_EPS)) {
            float pe1 = (float)(1.0 / (double)f);
            float u = pe1 * dot3(px, py, pz, dt[0], dt[1], dt[2]);
            float v = pe1 * dot3(rmd[0], rmd[1], rmd[2], dq[0], dq[1], dq[2]);
            float w = pe1 * s->dw[t];
            if ((w < d) && !(((double)u < ORC_EPS) || ((double)v < ORC_EPS) ||
                             ((double)(u + v) > 1 + ORC_EPS) || ((double)w < ORC_EPS))) {
                cnt[ORC_CNT_ACCEPT]++;
                d = w;
                out->rmi = t;
                out->d = w;
                for (int k = 0; k < 3; k++) {
                    out->rad[k] = s->rad[3 * (size_t)t + k];
                    out->pnt[k] = d * rmd[k];
                    out->nrm[k] = s->nrm[3 * (size_t)t + k];
                }
            }
        }
    }
    cnt[ORC_CNT_LEAF] += s->ntri;
}

int orc_render(const orc_scene* s, const float xform[12], int mode, int32_t row0,
               int32_t row1, uint32_t* argb, int64_t* hit, uint64_t counters[ORC_CNT_N],
               int nthreads) {
    return orc_render_ex(s, xform, mode, 0, row0, row1, argb, hit, counters, nthreads);
}

int orc_render_ex(const orc_scene* s, const float xform[12], int mode, int flags, int32_t row0,
                  int32_t row1, uint32_t* argb, int64_t* hit, uint64_t counters[ORC_CNT_N],
                  int nthreads) {
    static const float ident[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const float* X = xform ? xform : ident;
    const int32_t w = s->cam.w;
    if (row0 < 0) row0 = 0;
    if (row1 > s->cam.h) row1 = s->cam.h;
    if (mode == 0 && !s->bo) return -2;
    if ((flags & ORC_FLAG_SHADOW) && mode != 0) return -3;
    int status = 0;
    uint64_t tot[ORC_CNT_N] = {0};
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        uint64_t cnt[ORC_CNT_N] = {0};
        int st = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int32_t iy = row0; iy < row1; iy++) {
            for (int32_t ix = 0; ix < w; ix++) {
                int64_t i = (int64_t)iy * w + ix;
                float rmd[3];
                orc_primary_ray(&s->cam, ix, iy, rmd);
                orc_hit h;
                if (mode == 0) {
                    if (trace_kd(s, X, rmd, &h, cnt) != 0) st = -1;
                } else {
                    trace_flat(s, rmd, &h, cnt);
                }
                /* set_cam_cuda then color_cam_cuda (TD/Camera.cu:12-18,77-82) */
                uint32_t c = ORC_BG;
                if (h.rmi >= 0) {
                    cnt[ORC_CNT_HITPIX]++;
                    c = orc_phong(h.pnt, h.nrm, rmd, h.rad);
                    if (flags & ORC_FLAG_SHADOW) {
                        float sd[3], odl[3], Lmax;
                        shadow_ray(&h, sd, odl, &Lmax);
                        int sh = trace_shadow(s, sd, odl, Lmax, h.rmi, cnt);
                        if (sh < 0) st = -1;
                        if (sh > 0) c = 0x00000000u;
                    }
                }
                if (argb) argb[i] = c;
                if (hit) hit[i] = h.rmi;
            }
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            for (int k = 0; k < ORC_CNT_N; k++) {
                if (k == ORC_CNT_MAXSTACK) { if (cnt[k] > tot[k]) tot[k] = cnt[k]; }
                else tot[k] += cnt[k];
            }
            if (st) status = st;
        }
    }
    if (counters)
        for (int k = 0; k < ORC_CNT_N; k++) counters[k] = tot[k];
    (void)nthreads;
    return status;
}

/* The reference's window buffer across frames (TD/WinMain.cpp:174-239).  The
 * u32 buffer persists from frame to frame; init_cam_mem_cuda zeroes it
 * (TD/Camera.cu:98).  Each frame after intersect:
 *   color_pixels(PHONG_COLOR_TAG) -> color_cam_cuda writes only the pixels
 *     whose rmi >= 0 (TD/Camera.cu:27-61, :81), D2H (:84), blit
 *     (TD/WinMain.cpp:213-217): that is the displayed frame;
 *   color_pixels(SET_COLOR_TAG) -> set_cam_cuda fills the background and,
 *     the `break` missing, color_cam_cuda runs again (TD/Camera.cu:77-82):
 *     the buffer is this frame's clean frame (background + Phong).
 * `window` (npix, zero before the first frame) is that buffer; `clean` and
 * `hit` are the frame's steady-state render (orc_render); `displayed`
 * receives what the window shows. */
void orc_window_frame(uint32_t* window, const uint32_t* clean, const int64_t* hit, int64_t npix,
                      uint32_t* displayed) {
    for (int64_t i = 0; i < npix; i++)
        if (hit[i] >= 0) window[i] = clean[i];
    memcpy(displayed, window, sizeof(uint32_t) * (size_t)npix);
    for (int64_t i = 0; i < npix; i++) window[i] = hit[i] >= 0 ? clean[i] : ORC_BG;
}

/* Per-pixel pop counts (interior + leaf) of the KD traversal: a workload
 * profile for the kernels' load balance (not part of the reference). */
int orc_pixel_visits(const orc_scene* s, const float xform[12], uint32_t* visits, int nthreads) {
    static const float ident[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const float* X = xform ? xform : ident;
    if (!s->bo) return -2;
    const int32_t w = s->cam.w, h = s->cam.h;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int32_t iy = 0; iy < h; iy++)
        for (int32_t ix = 0; ix < w; ix++) {
            uint64_t cnt[ORC_CNT_N] = {0};
            float rmd[3];
            orc_hit hh;
            orc_primary_ray(&s->cam, ix, iy, rmd);
            trace_kd(s, X, rmd, &hh, cnt);
            visits[(int64_t)iy * w + ix] = (uint32_t)(cnt[ORC_CNT_INTERIOR] + cnt[ORC_CNT_LEAF]);
        }
    (void)nthreads;
    return 0;
}
