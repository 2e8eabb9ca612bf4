/* tools/sched_sim.c -- design tool (not product, not a test): simulates
 * kernel 3's per-wave item pool on the CPU with the oracle's arithmetic and
 * compares pop policies by pool iterations per unit (the chain of a wave)
 * and in total (the wave-iterations the GPU issues).
 *
 *   gcc -O2 -ffp-contract=off -fopenmp -o /tmp/sched_sim tools/sched_sim.c -lm
 *   /tmp/sched_sim mesh.ply W H loader_mode rays_per_unit cap policy
 *
 * Policies (every one visits the same items; only their order differs):
 *   0  LIFO: pop the top min(n, 128, cap - slack - n) items (kernel 3, r02)
 *   1  FIFO: the same count from the bottom (oldest first), a single LIFO pop
 *      when there is no room (the DFS bound of the fallback needs LIFO)
 *   2  shallowest first: the same count, the items of least depth (a bound:
 *      a priority pool, not cheap on the GPU)
 *   3  split FIFO: half from the bottom, half from the top
 * Children are pushed as the kernel pushes them: per popped slot (lanes
 * 0-63, then 64-127) all first children, then all second ones.
 */
#include "../oracle/oracle.c"

typedef struct { int32_t ref; float t0, t1; int ray; int depth; } item_t;

static int slab_cmp(const orc_scene* s, const float r[3], int32_t cni, float* maxt0, float* mint1) {
    const float* b = s->bo + 6 * (int64_t)cni;
    float rx = r[0], ry = r[1], rz = r[2];
    float t0x = rx > 0 ? b[0] * (1 / rx) : b[3] * (1 / rx);
    float t1x = rx > 0 ? b[3] * (1 / rx) : b[0] * (1 / rx);
    float t0y = ry > 0 ? b[1] * (1 / ry) : b[4] * (1 / ry);
    float t1y = ry > 0 ? b[4] * (1 / ry) : b[1] * (1 / ry);
    float t0z = rz > 0 ? b[2] * (1 / rz) : b[5] * (1 / rz);
    float t1z = rz > 0 ? b[5] * (1 / rz) : b[2] * (1 / rz);
    *maxt0 = fmaxf(t0z + 0 / rz, fmaxf(t0x + 0 / rx, t0y + 0 / ry));
    *mint1 = fminf(t1z + 0 / rz, fminf(t1x + 0 / rx, t1y + 0 / ry));
    return (double)*mint1 >= (double)*maxt0 - ORC_EPS && (double)*maxt0 > -ORC_EPS;
}

/* children of interior item it that the reference visits (slab-passed or
 * leaf), first then second (TD/Trixel.cu:146-170) */
static int expand_sim(const orc_scene* s, const float r[3], item_t it, item_t out[2]) {
    int32_t c = it.ref;
    const uint8_t* cf = s->cut + 3 * (int64_t)c;
    float dir = (r[0] * cf[0]) + (r[1] * cf[1]) + (r[2] * cf[2]);
    float mx0 = it.t0 * dir, mn1 = it.t1 * dir;
    float s1 = (float)((double)s->s1[c] + ORC_EPS), s2 = s->s2[c];
    int32_t L = (int32_t)s->left[c], R = (int32_t)s->right[c], first, second = -1;
    if ((double)mx0 < (double)s2 + ORC_EPS) {
        first = L;
        if ((double)mn1 > (double)s2 - ORC_EPS) second = R;
    } else {
        first = R;
        if (mn1 < s1 || mx0 < s1) second = L;
    }
    int n = 0;
    float a = 0, b = 0;
    if (s->is_leaf[first] || slab_cmp(s, r, first, &a, &b)) out[n++] = (item_t){first, a, b, it.ray, it.depth + 1};
    a = b = 0;
    if (second >= 0 && (s->is_leaf[second] || slab_cmp(s, r, second, &a, &b)))
        out[n++] = (item_t){second, a, b, it.ray, it.depth + 1};
    return n;
}

static int cmp_depth(const void* a, const void* b) {
    const item_t *x = (const item_t*)a, *y = (const item_t*)b;
    return x->depth - y->depth;
}

static int cmp_ll(const void* a, const void* b) {
    long long x = *(const long long*)a, y = *(const long long*)b;
    return x < y ? -1 : x > y;
}

typedef struct {
    const orc_scene* s;
    const orc_camera* cam;
    int w, h, ux, uh, uw, rays, cap, slack;
} ctx_t;

/* Rays of unit u into rr[base..base+rays) and its root items onto st; returns the new pool size. */
static long long seed_unit(const ctx_t* C, long long u, float rr[][3], int base, item_t* st, long long nst) {
    for (int l = 0; l < C->rays; l++) {
        int x = (int)(u % C->ux) * C->uw + (l % C->uw), y = (int)(u / C->ux) * C->uh + (l / C->uw);
        if (x >= C->w || y >= C->h) continue;
        orc_primary_ray(C->cam, x, y, rr[base + l]);
        float a, b;
        if (C->s->is_leaf[0]) { st[nst++] = (item_t){0, 0, 0, base + l, 0}; continue; }
        if (slab_cmp(C->s, rr[base + l], 0, &a, &b)) st[nst++] = (item_t){0, a, b, base + l, 0};
    }
    return nst;
}

/* One LIFO pool iteration over st (take <= per); returns the new size and counts pops per slot group. */
static long long step(const ctx_t* C, float rr[][3], item_t* st, long long nst, int per, long long* items) {
    item_t pop[256], kid1[256], kid2[256];
    long long take = nst < per ? nst : per;
    if (take > C->cap - C->slack - nst) take = C->cap - C->slack - nst;
    if (take < 1) take = 1;
    for (int k = 0; k < take; k++) pop[k] = st[nst - take + k];
    nst -= take;
    for (int sl = 0; sl * 64 < take; sl++) {
        int n1 = 0, n2 = 0;
        for (int k = sl * 64; k < take && k < sl * 64 + 64; k++) {
            item_t it = pop[k];
            (*items)++;
            int32_t c = it.ref;
            if (C->s->is_leaf[c]) continue;
            const float* r = rr[it.ray];
            const uint8_t* cf = C->s->cut + 3 * (int64_t)c;
            float dir = (r[0] * cf[0]) + (r[1] * cf[1]) + (r[2] * cf[2]);
            float mx0 = it.t0 * dir, mn1 = it.t1 * dir;
            float s1 = (float)((double)C->s->s1[c] + ORC_EPS), s2 = C->s->s2[c];
            int32_t L = (int32_t)C->s->left[c], R = (int32_t)C->s->right[c], first, second = -1;
            if ((double)mx0 < (double)s2 + ORC_EPS) {
                first = L;
                if ((double)mn1 > (double)s2 - ORC_EPS) second = R;
            } else {
                first = R;
                if (mn1 < s1 || mx0 < s1) second = L;
            }
            float a = 0, b = 0;
            if (C->s->is_leaf[first] || slab_cmp(C->s, r, first, &a, &b))
                kid1[n1++] = (item_t){first, a, b, it.ray, it.depth + 1};
            a = b = 0;
            if (second >= 0 && (C->s->is_leaf[second] || slab_cmp(C->s, r, second, &a, &b)))
                kid2[n2++] = (item_t){second, a, b, it.ray, it.depth + 1};
        }
        for (int k = 0; k < n1; k++) st[nst++] = kid1[k];
        for (int k = 0; k < n2; k++) st[nst++] = kid2[k];
    }
    return nst;
}

static double tl_cost = 1.6;
static int cmp_dbl(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

typedef struct { long long cost, unit; } cu_t;
static int cmp_cu(const void* a, const void* b) {
    const cu_t *x = (const cu_t*)a, *y = (const cu_t*)b;
    return x->cost < y->cost ? 1 : x->cost > y->cost ? -1 : (x->unit > y->unit) - (x->unit < y->unit);
}

/* Wave schedules over the traced units in cost order (heaviest first):
 *   mode 1 (pairs): wave k holds units k and k + m/2 in one pool from the start
 *   mode 2 (refill): wave k takes units k, k + W, k + 2W, ... (W waves); two
 *                    slots of `rays` rays; a drained slot takes the next unit */
static void waves(const ctx_t* C, const cu_t* order, long long m, int mode, long long W) {
    long long nw = mode == 1 ? (m + 1) / 2 : W;
    long long* chain = (long long*)calloc((size_t)nw, sizeof(long long));
    long long tot = 0, items = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : tot, items)
    for (long long k = 0; k < nw; k++) {
        item_t* st = (item_t*)malloc(sizeof(item_t) * 8192);
        float rr[128][3];
        long long nst = 0, it = 0, next = k;
        long long inslot[2] = {0, 0};
        int live[2] = {0, 0};
        if (mode == 1) {
            nst = seed_unit(C, order[k].unit, rr, 0, st, nst);
            if (k + nw < m) nst = seed_unit(C, order[k + nw].unit, rr, C->rays, st, nst);
            while (nst > 0) { nst = step(C, rr, st, nst, 128, &items); it++; }
        } else {
            for (int sl = 0; sl < 2; sl++)
                if (next < m) { long long b = nst; nst = seed_unit(C, order[next].unit, rr, sl * C->rays, st, nst); inslot[sl] = nst - b; live[sl] = 1; next += W; }
            while (nst > 0 || live[0] || live[1]) {
                if (nst > 0) { nst = step(C, rr, st, nst, 128, &items); it++; }
                for (int sl = 0; sl < 2; sl++) {
                    long long c = 0;
                    for (long long q = 0; q < nst; q++) c += st[q].ray / C->rays == sl;
                    if (live[sl] && c == 0) {
                        live[sl] = 0;
                        if (next < m) { nst = seed_unit(C, order[next].unit, rr, sl * C->rays, st, nst); live[sl] = 1; next += W; }
                    }
                }
            }
        }
        chain[k] = it;
        tot += it;
        free(st);
    }
    qsort(chain, (size_t)nw, sizeof(long long), cmp_ll);
    printf("  schedule %s (%lld waves): wave-iterations %lld (%.1f items each); chain median %lld p99 %lld max %lld\n",
           mode == 1 ? "pairs" : "refill", nw, tot, (double)items / (double)tot, chain[nw / 2], chain[nw * 99 / 100], chain[nw - 1]);
    free(chain);
}

int main(int argc, char** argv) {
    const char* mesh = argc > 1 ? argv[1] : "/tmp/knot.ply";
    int w = argc > 2 ? atoi(argv[2]) : 1920, h = argc > 3 ? atoi(argv[3]) : 1080;
    int mode = argc > 4 ? atoi(argv[4]) : 0;
    int rays = argc > 5 ? atoi(argv[5]) : 16;
    int cap = argc > 6 ? atoi(argv[6]) : 352;
    int policy = argc > 7 ? atoi(argv[7]) : 0;
    const char* tm = getenv("TWO_MAX");
    const int two_max = tm ? atoi(tm) : 32;
    const char* tm3 = getenv("THREE_MAX");
    const int three_max = tm3 ? atoi(tm3) : 8;
    const char* tcs = getenv("TL_COST");
    tl_cost = tcs ? atof(tcs) : 1.6;
    /* BLOCK_WAVES=W: a block of W waves pops one shared pool (W x 128 items
     * per iteration; cap is then the block's pool) */
    const char* bws = getenv("BLOCK_WAVES");
    const int bw = bws ? atoi(bws) : 1;
    float* pts; uint32_t n; orc_leaf* lf;
    if (orc_read_ply(mesh, mode, &pts, &n, &lf)) { fprintf(stderr, "read fail\n"); return 1; }
    orc_node* nodes = (orc_node*)malloc(sizeof(orc_node) * (2 * (size_t)n - 1));
    orc_build_kd(lf, n, nodes);
    int height = 0;
    for (uint32_t m = 1; m < n; m *= 2) height++;
    const int slack = height + 2;
    /* deepest node depth whose children are all interior: floor(n / 2^(d+1)) >= 2 */
    int dmax = -1;
    while ((n >> (dmax + 2)) >= 2) dmax++;
    printf("ntri %u height %d two-level dmax %d two_max %d\n", n, height, dmax, two_max);
    float* rad = (float*)malloc(sizeof(float) * 3 * n);
    for (uint32_t i = 0; i < 3 * n; i++) rad[i] = 0.5f;
    orc_camera cam;
    const float pos[3] = {0, 0.1f, -1}, la[3] = {0, 0.1f, 0}, up[3] = {0, 1, 0};
    orc_camera_basis(w, h, orc_film_w(w, h), 0.024f, 0.055f, pos, la, up, &cam);
    orc_scene* s = orc_scene_create(pts, rad, n, nodes, &cam);
    const int uw = rays < 8 ? rays : 8, uh = rays / uw;  // unit: uw x uh pixels
    const int ux = (w + uw - 1) / uw, uy = (h + uh - 1) / uh;
    const long long nu = (long long)ux * uy;
    long long* iters_of = (long long*)calloc((size_t)nu, sizeof(long long));
    long long tot_items = 0, tot_iters = 0, peak = 0, mixed = 0, slots = 0, tot2 = 0, tot2s = 0;
    double* cost_of = (double*)calloc((size_t)nu, sizeof(double));
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : tot_items, tot_iters, mixed, slots, tot2, tot2s) reduction(max : peak)
    for (long long u = 0; u < nu; u++) {
        item_t* st = (item_t*)malloc(sizeof(item_t) * 16384);
        item_t pop[128 * 8], kid1[128], kid2[128];
        float rr[64][3];
        long long nst = 0, iters = 0, items = 0, iters2 = 0, iters_two_slot = 0;
        for (int l = 0; l < rays; l++) {
            int x = (int)(u % ux) * uw + (l % uw), y = (int)(u / ux) * uh + (l / uw);
            if (x >= w || y >= h) continue;
            orc_primary_ray(&cam, x, y, rr[l]);
            float a, b;
            if (s->is_leaf[0]) { st[nst++] = (item_t){0, 0, 0, l, 0}; continue; }
            if (slab_cmp(s, rr[l], 0, &a, &b)) st[nst++] = (item_t){0, a, b, l, 0};
        }
        while (nst > 0) {
            if (policy == 5 && nst <= three_max) {
                /* three-level iteration (8 lanes per item): the item's node,
                 * its children and grandchildren visited in one iteration,
                 * great-grandchildren pushed; nodes deeper than the implicit
                 * levels stop the expansion there */
                int npop = (int)nst;
                for (int k = 0; k < npop; k++) pop[k] = st[k];
                nst = 0;
                iters++;
                iters2++;
                for (int k = 0; k < npop; k++) {
                    item_t lvl[8], nxt[8];
                    int nl = 1;
                    lvl[0] = pop[k];
                    for (int L = 0; L < 3 && nl; L++) {
                        int nn = 0;
                        for (int q = 0; q < nl; q++) {
                            item_t it = lvl[q];
                            items++;
                            if (s->is_leaf[it.ref]) continue;
                            item_t kids[2];
                            int nkid = expand_sim(s, rr[it.ray], it, kids);
                            /* children are visited in this iteration only while
                             * their parent lies in the implicit levels */
                            for (int r2 = 0; r2 < nkid; r2++) {
                                if (L < 2 && it.depth <= dmax && !s->is_leaf[kids[r2].ref]) nxt[nn++] = kids[r2];
                                else st[nst++] = kids[r2];
                            }
                        }
                        for (int q = 0; q < nn; q++) lvl[q] = nxt[q];
                        nl = nn;
                        if (L == 2) break;
                    }
                    (void)nl;
                }
                if (nst > peak) peak = nst;
                continue;
            }
            if ((policy == 4 || policy == 5 || policy == 6) && nst <= two_max) {
                /* two-level iteration: item k on lane k (its node's record) and
                 * lane k + 32 (its children's records, implicit BFS positions):
                 * children of an eligible node are expanded in the same
                 * iteration, grandchildren pushed */
                int npop = (int)nst, nk = 0;
                for (int k = 0; k < npop; k++) pop[k] = st[k];
                nst = 0;
                iters++;
                iters2++;
                for (int k = 0; k < npop; k++) {
                    item_t it = pop[k];
                    items++;
                    if (s->is_leaf[it.ref]) continue;
                    item_t kids[2];
                    int nkid = expand_sim(s, rr[it.ray], it, kids);
                    for (int q = 0; q < nkid; q++) {
                        if (policy == 6 && s->is_leaf[kids[q].ref]) {
                            items++;  /* heap layout: a leaf child's MT test in this iteration */
                        } else if ((it.depth <= dmax || policy == 6) && !s->is_leaf[kids[q].ref]) {
                            item_t g[2];
                            items++;
                            int ng = expand_sim(s, rr[it.ray], kids[q], g);
                            for (int r2 = 0; r2 < ng; r2++) st[nst++] = g[r2];
                        } else {
                            st[nst++] = kids[q];
                        }
                    }
                    (void)nk;
                }
                if (nst > peak) peak = nst;
                continue;
            }
            long long take = nst < 128 * bw ? nst : 128 * bw;
            if (take > cap - slack - nst) take = cap - slack - nst;
            int lifo = policy == 0 || policy >= 4;
            if (take < 1) { take = 1; lifo = 1; }
            if (lifo) {
                for (int k = 0; k < take; k++) pop[k] = st[nst - take + k];
                nst -= take;
            } else if (policy == 1) {
                for (int k = 0; k < take; k++) pop[k] = st[k];
                memmove(st, st + take, sizeof(item_t) * (size_t)(nst - take));
                nst -= take;
            } else if (policy == 2) {
                qsort(st, (size_t)nst, sizeof(item_t), cmp_depth);
                for (int k = 0; k < take; k++) pop[k] = st[k];
                memmove(st, st + take, sizeof(item_t) * (size_t)(nst - take));
                nst -= take;
            } else {
                long long hb = take / 2, ht = take - hb;
                for (int k = 0; k < hb; k++) pop[k] = st[k];
                for (int k = 0; k < ht; k++) pop[hb + k] = st[nst - ht + k];
                memmove(st, st + hb, sizeof(item_t) * (size_t)(nst - take));
                nst -= take;
            }
            iters++;
            if (take > 64) iters_two_slot++;
            for (int sl = 0; sl < 2 * bw; sl++) {
                int n1 = 0, n2 = 0, nleaf = 0, nint = 0;
                for (int k = sl * 64; k < take && k < sl * 64 + 64; k++) {
                    item_t it = pop[k];
                    items++;
                    int32_t c = it.ref;
                    if (s->is_leaf[c]) { nleaf++; continue; }
                    nint++;
                    const float* r = rr[it.ray];
                    const uint8_t* cf = s->cut + 3 * (int64_t)c;
                    float dir = (r[0] * cf[0]) + (r[1] * cf[1]) + (r[2] * cf[2]);
                    float mx0 = it.t0 * dir, mn1 = it.t1 * dir;
                    float s1 = (float)((double)s->s1[c] + ORC_EPS), s2 = s->s2[c];
                    int32_t L = (int32_t)s->left[c], R = (int32_t)s->right[c], first, second = -1;
                    if ((double)mx0 < (double)s2 + ORC_EPS) {
                        first = L;
                        if ((double)mn1 > (double)s2 - ORC_EPS) second = R;
                    } else {
                        first = R;
                        if (mn1 < s1 || mx0 < s1) second = L;
                    }
                    float a = 0, b = 0;
                    if (s->is_leaf[first] || slab_cmp(s, r, first, &a, &b))
                        kid1[n1++] = (item_t){first, a, b, it.ray, it.depth + 1};
                    a = b = 0;
                    if (second >= 0 && (s->is_leaf[second] || slab_cmp(s, r, second, &a, &b)))
                        kid2[n2++] = (item_t){second, a, b, it.ray, it.depth + 1};
                }
                if (nleaf || nint) slots++;
                if (nleaf && nint) mixed++;
                for (int k = 0; k < n1; k++) st[nst++] = kid1[k];
                for (int k = 0; k < n2; k++) st[nst++] = kid2[k];
            }
            if (nst > peak) peak = nst;
        }
        iters_of[u] = iters;
        /* relative iteration latencies: one slot 1.0, two slots 1.3, two-level 1.6 */
        cost_of[u] = (double)(iters - iters2 - iters_two_slot) + 1.3 * (double)iters_two_slot + tl_cost * (double)iters2;
        tot2 += iters2;
        tot2s += iters_two_slot;
        tot_items += items;
        tot_iters += iters;
        free(st);
    }
    long long nz = 0;
    cu_t* order = (cu_t*)malloc(sizeof(cu_t) * (size_t)nu);
    for (long long u = 0; u < nu; u++) if (iters_of[u]) { order[nz] = (cu_t){iters_of[u], u}; iters_of[nz++] = iters_of[u]; }
    qsort(order, (size_t)nz, sizeof(cu_t), cmp_cu);
    qsort(iters_of, (size_t)nz, sizeof(long long), cmp_ll);
    printf("policy %d rays %d cap %d: units traced %lld, items %lld, wave-iterations %lld (%.1f items each), "
           "peak pool %lld, mixed slots %.3f\n", policy, rays, cap, nz, tot_items, tot_iters,
           (double)tot_items / (double)(tot_iters ? tot_iters : 1), peak, (double)mixed / (double)(slots ? slots : 1));
    printf("  chain (iterations per unit): median %lld p90 %lld p99 %lld p99.9 %lld max %lld; top-16:",
           iters_of[nz / 2], iters_of[nz * 9 / 10], iters_of[nz * 99 / 100], iters_of[nz * 999 / 1000], iters_of[nz - 1]);
    for (long long k = nz - 16; k < nz; k++) if (k >= 0) printf(" %lld", iters_of[k]);
    printf("\n");
    {
        double tc = 0, mc = 0;
        for (long long u = 0; u < nu; u++) { tc += cost_of[u]; if (cost_of[u] > mc) mc = cost_of[u]; }
        qsort(cost_of, (size_t)nu, sizeof(double), cmp_dbl);
        printf("  two-level iterations %lld, two-slot %lld; cost (1 / 1.3 / 1.6 per one-slot / two-slot / two-level): "
               "total %.0f, p99.9 %.1f, max %.1f\n", tot2, tot2s, tc, cost_of[nu * 999 / 1000], mc);
    }
    ctx_t C = {s, &cam, w, h, ux, uh, uw, rays, cap, slack};
    if (argc > 8) {
        waves(&C, order, nz, 1, 0);
        for (int k = 8; k < argc; k++) waves(&C, order, nz, 2, atoll(argv[k]));
    }
    return 0;
}
