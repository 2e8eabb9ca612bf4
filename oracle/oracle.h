/*
 * oracle/oracle.h -- CPU restatement of the reference ray-cast hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in cpp_cuda_raytracer_dev_amd/ may link,
 * import or call this library: it is the parity checker used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 *
 * Parity status: "parity unpinned" against the reference binary -- the
 * reference (ams3878/cpp_cuda_raytracer_dev) ships no tests, no golden
 * vectors, and compiling/running it in this environment was denied (SURVEY.md
 * §8c).  This restatement is pinned instead against (1) an independent numpy
 * restatement (oracle/np_oracle.py) on small scenes, (2) hand-derived
 * known-answer tests (tests/test_oracle_kat.py) and (3) structural invariants
 * of the KD tree.  See DESIGN.md §Parity.
 *
 * Every function cites the reference file:line it restates
 * (TD/ = TEST_Dungeonrun/ in the reference tree).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* kd_leaf_sort (TD/Trixel.h:20-30): a per-triangle AABB plus its position in
 * each of the six sorted lists. */
typedef struct orc_leaf {
    float x0, x1, y0, y1, z0, z1;
    int64_t sx0, sy0, sz0, sx1, sy1, sz1;
    int64_t tri;
} orc_leaf;

/* kd_tree_node (TD/Trixel.h:68-79), world space. */
typedef struct orc_node {
    float x0, x1, y0, y1, z0, z1;
    float s1, s2;
    int32_t cut_flag;
    int32_t is_leaf;
    int64_t tri_index, left, right, parent;
    int64_t l, m, r;
} orc_node;

/* Camera basis produced by Camera::Camera (TD/Camera.cpp:5-117). */
typedef struct orc_camera {
    int32_t w, h;
    float pos[3];
    float n[3], u[3], v[3];
    float n_mod[3], u_mod[3], v_mod[3];
    float pix_w, pix_h;
} orc_camera;

/* Counters for the roofline model. */
enum {
    ORC_CNT_INTERIOR = 0, /* interior pops (V_int)                    */
    ORC_CNT_LEAF = 1,     /* leaf pops (V_leaf)                        */
    ORC_CNT_ACCEPT = 2,   /* accepted MT hits, every write event (H)   */
    ORC_CNT_HITPIX = 3,   /* pixels with a final hit                   */
    ORC_CNT_DESCEND = 4,  /* interior pops that passed the slab test   */
    ORC_CNT_MAXSTACK = 5, /* max stack occupancy seen                  */
    ORC_CNT_N = 6
};

/* read_ply (TD/read_ply.cpp:13-152).  mode: 0 = "x y z", 1 = "x y z c i",
 * 2 = "x y z nx ny nz".  Accepts the reference's "end_header" header and the
 * headerless "[ply\n]nv\nnf\n" prelude used by tester.ply / dump*.ply (H9).
 * Outputs are malloc'd; free with orc_free.  Returns 0 or a negative error. */
int orc_read_ply(const char* path, int mode, float** points9, uint32_t* ntri,
                 orc_leaf** leafs);

/* The face-assembly half of read_ply from an indexed mesh (arity 3 or 4 per
 * face, `arity[f]`, indices flattened in `idx`). */
int orc_assemble(const float* verts, int64_t nvert, const int32_t* arity,
                 const int32_t* idx, int64_t nface, float** points9,
                 uint32_t* ntri, orc_leaf** leafs);

void orc_free(void* p);

/* merge_sort (TD/sort.h:11-60) on one of the six keys (1..6 = x0,y0,z0,x1,y1,z1). */
void orc_merge_sort(orc_leaf* list, orc_leaf* work, uint32_t n, int key);

/* set_sorted_voxels + create_kd (TD/Trixel.h:135-473), literal.  `nodes`
 * must hold 2*ntri-1 entries. */
int orc_build_kd(const orc_leaf* leafs, uint32_t ntri, orc_node* nodes);

/* Camera::Camera basis (TD/Camera.cpp:5-67). */
void orc_camera_basis(int32_t w, int32_t h, float f_w, float f_h, float focal,
                      const float pos[3], const float la[3], const float up[3],
                      orc_camera* cam);

/* WinMain's film width: ((float)w / h) * .024f (TD/WinMain.cpp:29,69-70). */
float orc_film_w(int32_t w, int32_t h);

/* The fast inverse square roots (TD/vector.cpp:13-26 host, 8 steps;
 * TD/vector.cuh:79-95 device, 21 steps). */
float orc_host_vector_norm(float s);
float orc_device_inverse_sqrt(float x, float y, float z);

/* A rendered scene: triangle SoA (TD/Trixel.cu:11-36) and camera-relative
 * node arrays (TD/Camera.cu:137-162). */
typedef struct orc_scene orc_scene;
orc_scene* orc_scene_create(const float* points9, const float* rad3,
                            uint32_t ntri, const orc_node* nodes,
                            const orc_camera* cam);
void orc_scene_destroy(orc_scene* s);

/* Render rows [row0, row1) of the frame: bg fill -> intersect -> Phong, the
 * steady-state frame of TD/WinMain.cpp:212-237.  mode 0 = KD traversal
 * (intersect_voxel_cuda), 1 = flat list (intersect_trixel_cuda).  argb / hit
 * are full-frame arrays (w*h); only the requested rows are written.
 * xform = rot_m rows (x.i x.j x.k x.w, y..., z...), identity in every config.
 * nthreads <= 0: OpenMP default.  Returns 0, or -1 on a stack overflow. */
int orc_render(const orc_scene* s, const float xform[12], int mode,
               int32_t row0, int32_t row1, uint32_t* argb, int64_t* hit,
               uint64_t counters[ORC_CNT_N], int nthreads);

/* orc_render with flags.  ORC_FLAG_SHADOW (KD mode only): one shadow ray
 * per hit pixel (definition in oracle.c trace_shadow);
 * shadowed pixels are 0x00000000 and the shadow rays' visits are added to
 * the same counters.  Returns -3 for shadow with mode 1. */
#define ORC_FLAG_SHADOW 4
int orc_render_ex(const orc_scene* s, const float xform[12], int mode, int flags,
                  int32_t row0, int32_t row1, uint32_t* argb, int64_t* hit,
                  uint64_t counters[ORC_CNT_N], int nthreads);

/* One primary ray (init_cam_mem_cuda, TD/Camera.cu:103-104). */
void orc_primary_ray(const orc_camera* cam, int32_t ix, int32_t iy, float out[3]);

/* The reference's persistent window buffer for one frame (oracle.c): the
 * displayed frame (ghosting under motion) from `window` (zero before the
 * first frame) and the frame's clean render; `window` becomes the clean frame. */
void orc_window_frame(uint32_t* window, const uint32_t* clean, const int64_t* hit, int64_t npix,
                      uint32_t* displayed);

/* Per-pixel visit counts (interior + leaf pops) of the KD traversal. */
int orc_pixel_visits(const orc_scene* s, const float xform[12], uint32_t* visits, int nthreads);

/* Phong of one hit (color_cam_cuda, TD/Camera.cu:27-60). */
uint32_t orc_phong(const float pnt[3], const float nrm[3], const float rmd[3],
                   const float rad[3]);

#ifdef __cplusplus
}
#endif
#endif
