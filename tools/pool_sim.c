/* tools/pool_sim.c -- design tool (not product, not a test): simulates the
 * wave-cooperative traversal on the CPU with the oracle's arithmetic to size
 * its shared LDS item stack.  For every 8x8-pixel wave tile it runs the item
 * pool (pop min(n, 64) from the top, expand, push children) and reports the
 * pool's peak size and iteration count against the per-lane DFS's max visits.
 *
 *   gcc -O2 -ffp-contract=off -fopenmp -o /tmp/pool_sim tools/pool_sim.c -lm
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

int main(int argc, char** argv) {
    const char* mesh = argc > 1 ? argv[1] : "/tmp/dragon.ply";
    int w = argc > 2 ? atoi(argv[2]) : 1920, h = argc > 3 ? atoi(argv[3]) : 1080;
    int mode = argc > 4 ? atoi(argv[4]) : 0;
    float* pts; uint32_t n; orc_leaf* lf;
    if (orc_read_ply(mesh, mode, &pts, &n, &lf)) { fprintf(stderr, "read fail\n"); return 1; }
    orc_node* nodes = (orc_node*)malloc(sizeof(orc_node) * (2 * (size_t)n - 1));
    orc_build_kd(lf, n, nodes);
    float* rad = (float*)malloc(sizeof(float) * 3 * n);
    for (uint32_t i = 0; i < 3 * n; i++) rad[i] = 0.5f;
    orc_camera cam;
    const float pos[3] = {0, 0.1f, -1}, la[3] = {0, 0.1f, 0}, up[3] = {0, 1, 0};
    orc_camera_basis(w, h, orc_film_w(w, h), 0.024f, 0.055f, pos, la, up, &cam);
    orc_scene* s = orc_scene_create(pts, rad, n, nodes, &cam);
    int tx = (w + 7) / 8, ty = (h + 7) / 8;
    long long tot_items = 0, tot_iters = 0, worst_iters = 0, worst_lane = 0, peak = 0, sum_lane_max = 0;
    static long long hist[64];
#pragma omp parallel for schedule(dynamic) reduction(+ : tot_items, tot_iters, sum_lane_max) \
    reduction(max : worst_iters, worst_lane, peak)
    for (int t = 0; t < tx * ty; t++) {
        item_t* st = (item_t*)malloc(sizeof(item_t) * 200000);
        float rays[64][3];
        int lane_visits[64] = {0};
        long long nst = 0, iters = 0, items = 0, mx = 0;
        for (int l = 0; l < 64; l++) {
            int x = (t % tx) * 8 + (l & 7), y = (t / tx) * 8 + (l >> 3);
            if (x >= w || y >= h) continue;
            orc_primary_ray(&cam, x, y, rays[l]);
            float a, b;
            if (s->is_leaf[0]) { st[nst++] = (item_t){0, 0, 0, l, 0}; continue; }
            if (slab_cmp(s, rays[l], 0, &a, &b)) st[nst++] = (item_t){0, a, b, l, 0};
        }
        while (nst > 0) {
            long long take = nst < 64 ? nst : 64;
            item_t pop[64];
            for (int k = 0; k < take; k++) pop[k] = st[nst - take + k];
            nst -= take;
            iters++;
            for (int k = 0; k < take; k++) {
                item_t it = pop[k];
                items++;
                lane_visits[it.ray]++;
                int32_t c = it.ref;
                if (s->is_leaf[c]) continue;
                const float* r = rays[it.ray];
                const uint8_t* cf = s->cut + 3 * (int64_t)c;
                float dir = (r[0] * cf[0]) + (r[1] * cf[1]) + (r[2] * cf[2]);
                float mx0 = it.t0 * dir, mn1 = it.t1 * dir;
                float s1 = (float)((double)s->s1[c] + ORC_EPS), s2 = s->s2[c];
                int32_t L = (int32_t)s->left[c], R = (int32_t)s->right[c], kids[2];
                int nk = 0;
                if ((double)mx0 < (double)s2 + ORC_EPS) {
                    if ((double)mn1 > (double)s2 - ORC_EPS) kids[nk++] = R;
                    kids[nk++] = L;
                } else {
                    if (mn1 < s1 || mx0 < s1) kids[nk++] = L;
                    kids[nk++] = R;
                }
                for (int q = 0; q < nk; q++) {
                    float a = 0, b = 0;
                    if (!s->is_leaf[kids[q]] && !slab_cmp(s, r, kids[q], &a, &b)) continue;
                    st[nst++] = (item_t){kids[q], a, b, it.ray, it.depth + 1};
                }
            }
            if (nst > mx) mx = nst;
        }
        int lm = 0;
        for (int l = 0; l < 64; l++) if (lane_visits[l] > lm) lm = lane_visits[l];
        tot_items += items; tot_iters += iters; sum_lane_max += lm;
        if (iters > worst_iters) worst_iters = iters;
        if (lm > worst_lane) worst_lane = lm;
        if (mx > peak) peak = mx;
#pragma omp critical
        hist[mx / 64 < 63 ? mx / 64 : 63]++;
        free(st);
    }
    printf("items %lld  pooled iterations %lld (worst tile %lld)  per-lane DFS: sum of wave max %lld (worst %lld)\n",
           tot_items, tot_iters, worst_iters, sum_lane_max, worst_lane);
    printf("peak pool size %lld items; tiles by peak/64:", peak);
    for (int k = 0; k < 64; k++) if (hist[k]) printf(" [%d]=%lld", k, hist[k]);
    printf("\n");
    return 0;
}
