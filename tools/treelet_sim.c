/* tools/treelet_sim.c -- design tool (not product, not a test): simulates the
 * wave-cooperative pool walk of kernel 3 on the CPU with the oracle's
 * arithmetic, for 16-ray units (8x2 pixels), pops of up to 128 items per
 * iteration under the kernel's capacity rule, with one-level items (a node's
 * child-box record: the current kernel) and two-level items (a node's
 * children and grandchildren in one record).  Reports iterations per unit.
 *
 *   gcc -O2 -ffp-contract=off -fopenmp -o /tmp/treelet_sim tools/treelet_sim.c -lm
 *   /tmp/treelet_sim /tmp/dragon.ply 1920 1080 0
 */
#include "../oracle/oracle.c"

typedef struct { int32_t ref; float t0, t1; int ray; } item_t;

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

/* children of interior node c visited by the reference (slab-passed or leaf) */
static int expand(const orc_scene* s, const float r[3], item_t it, item_t out[2]) {
    int32_t c = it.ref;
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
    int n = 0;
    for (int q = 0; q < nk; q++) {
        float a = 0, b = 0;
        if (!s->is_leaf[kids[q]] && !slab_cmp(s, r, kids[q], &a, &b)) continue;
        out[n++] = (item_t){kids[q], a, b, it.ray};
    }
    return n;
}

int main(int argc, char** argv) {
    const char* mesh = argc > 1 ? argv[1] : "/tmp/dragon.ply";
    int w = argc > 2 ? atoi(argv[2]) : 1920, h = argc > 3 ? atoi(argv[3]) : 1080;
    int mode = argc > 4 ? atoi(argv[4]) : 0;
    const int cap = argc > 5 ? atoi(argv[5]) : 384, per = argc > 6 ? atoi(argv[6]) : 128;
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
    const int tx = (w + 7) / 8, ty = (h + 1) / 2;
    for (int levels = 1; levels <= 2; levels++) {
        long long tot_iters = 0, worst = 0, items_all = 0, units = 0;
        long long hist[8] = {0};
#pragma omp parallel for schedule(dynamic) reduction(+ : tot_iters, items_all, units) reduction(max : worst)
        for (int t = 0; t < tx * ty; t++) {
            item_t* st = (item_t*)malloc(sizeof(item_t) * 100000);
            float rays[16][3];
            long long nst = 0, iters = 0, items = 0;
            for (int l = 0; l < 16; l++) {
                int x = (t % tx) * 8 + (l & 7), y = (t / tx) * 2 + (l >> 3);
                if (x >= w || y >= h) continue;
                orc_primary_ray(&cam, x, y, rays[l]);
                float a, b;
                if (s->is_leaf[0]) { st[nst++] = (item_t){0, 0, 0, l}; continue; }
                if (slab_cmp(s, rays[l], 0, &a, &b)) st[nst++] = (item_t){0, a, b, l};
            }
            if (nst == 0) { free(st); continue; }
            while (nst > 0) {
                long long take = nst < per ? nst : per;
                const long long room = levels == 1 ? cap - 22 - nst : (cap - 34 - nst) / 3;
                if (take > room) take = room;
                if (take < 1) take = 1;
                item_t pop[256];
                for (int k = 0; k < take; k++) pop[k] = st[nst - take + k];
                nst -= take;
                iters++;
                items += take;
                for (int k = 0; k < take; k++) {
                    item_t it = pop[k];
                    if (s->is_leaf[it.ref]) continue;
                    item_t c1[2];
                    int n1 = expand(s, rays[it.ray], it, c1);
                    for (int q = 0; q < n1; q++) {
                        if (levels == 2 && !s->is_leaf[c1[q].ref]) {
                            item_t c2[2];
                            int n2 = expand(s, rays[it.ray], c1[q], c2);
                            for (int z = 0; z < n2; z++) st[nst++] = c2[z];
                        } else {
                            st[nst++] = c1[q];
                        }
                    }
                }
            }
            tot_iters += iters;
            items_all += items;
            units++;
            if (iters > worst) worst = iters;
#pragma omp critical
            hist[iters / 16 < 7 ? iters / 16 : 7]++;
            free(st);
        }
        printf("levels %d: units %lld items %lld iterations %lld (mean %.1f, worst %lld) hist/16:", levels, units,
               items_all, tot_iters, (double)tot_iters / units, worst);
        for (int k = 0; k < 8; k++) printf(" %lld", hist[k]);
        printf("\n");
    }
    return 0;
}
