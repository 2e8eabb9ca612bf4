/*
 * rt_mi355x.h -- C ABI of the MI355X-native ray-cast hot path.
 *
 * Drop-in boundary for ams3878/cpp_cuda_raytracer_dev (TD/ = TEST_Dungeonrun/).
 * The reference's host objects (Camera, Trixel, Object, Quaternion) call the
 * device through free functions that return cudaError_t; each rt_* entry
 * point below names the reference function it replaces.  All functions
 * return RT_OK (0) or a negative rt_status; rt_last_error_string() explains
 * the last failure of the calling thread.  No torch types cross this ABI:
 * plain pointers, sizes and an optional hipStream_t passed as void*.
 *
 * Threading: one host thread per handle; handles are not thread-safe.
 * Rendering is stream-ordered; rt_read_frame synchronises.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 6): get-only option keys 10 and 11 are retired (rejected; they
 * were RT_OPT_COOP_USED and RT_OPT_FRAME_GROUP in round 4), RT_OPT_FAST_USED
 * moved to key 12 and became a bit mask, RT_OPT_ORDER_RESTORES is key 13. */
#define RT_ABI_VERSION 2

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,   /* bad argument / malformed input          */
    RT_ERR_HIP = -2,       /* a HIP runtime call failed                */
    RT_ERR_NOMEM = -3,     /* host or device allocation failed         */
    RT_ERR_IO = -4,        /* file could not be read / parsed          */
    RT_ERR_STATE = -5,     /* call out of order (e.g. render w/o tree) */
    RT_ERR_OVERFLOW = -6,  /* traversal stack overflow flagged by GPU  */
    RT_ERR_COMM = -7       /* RCCL missing or a collective call failed */
} rt_status;

/* Render modes: KD traversal (intersect_voxel_cuda, TD/Trixel.cu:41-172) or
 * the flat triangle list (intersect_trixel_cuda, TD/Trixel.cu:173-209). */
#define RT_MODE_KD 0u
#define RT_MODE_FLAT 1u

/* Render flags. */
#define RT_FLAG_WRITE_HIT 1u   /* also write the per-pixel hit triangle (d_rmi.index) */
#define RT_FLAG_COUNT 2u       /* accumulate traversal counters (rt_camera_counters)  */
/* One shadow ray per hit pixel (config C5; the reference's commented-out hook
 * at TD/Camera.cu:28-34).  The segment from the light (2,2,2) to the hit is
 * walked with the reference's traversal rules, entering a box only where the
 * segment enters it (entry parameter below Lmax, round 6); a pixel with an occluder
 * (any triangle but its own, w < 0.999*|segment|) is 0x00000000.  KD mode and
 * the wave-cooperative kernel only; the shadow rays'
 * visits are added to the same counters. */
#define RT_FLAG_SHADOW 4u
/* With a tile: write the tile's pixels at their frame positions in a w*h
 * buffer (argb and hit) instead of the packed band buffer; pixels of other
 * ranks' bands are not touched.  Rank 0 of a gather renders straight into
 * the frame it assembles (rt_comm_gather_frame with d_local == d_frame). */
#define RT_FLAG_FRAME_OUT 8u

/* Per-triangle AABB = kd_leaf (TD/Trixel.h:31-37); `tri` = tri_list_index. */
typedef struct rt_leaf_aabb {
    float x0, x1, y0, y1, z0, z1;
    int64_t tri;
} rt_leaf_aabb;

/* World-space tree node = Trixel::kd_tree::kd_tree_node (TD/Trixel.h:68-79),
 * BFS order, right = left + 1, 2*ntri-1 nodes. */
typedef struct rt_kd_node {
    float x0, x1, y0, y1, z0, z1; /* h_bound                            */
    float s1, s2;                 /* left child's max / right child's min on the cut axis */
    int32_t cut_flag;             /* 0 x1, 1 y1, 2 z1, 3 x0, 4 y0, 5 z0 */
    int32_t is_leaf;
    int64_t tri_index;            /* leaf: triangle; interior: -1       */
    int64_t left, right, parent;  /* leaf: -1, -1                       */
} rt_kd_node; /* 72 bytes */

/* Camera::o_prop basis (TD/Camera.h:32-42). */
typedef struct rt_camera_basis_t {
    float n[3], u[3], v[3];
    float n_mod[3], u_mod[3], v_mod[3];
    float pix_w, pix_h;
} rt_camera_basis_t;

/* Screen sharding: rows are cut into bands of 8; band b belongs to rank
 * b % nranks.  A rank renders its bands into a packed buffer of
 * rt_tile_packed_pixels() pixels (slot j = band rank + j*nranks). */
typedef struct rt_tile {
    int32_t nranks;
    int32_t rank;
} rt_tile;

typedef struct rt_scene rt_scene;   /* Trixel: triangles + KD tree on one device */
typedef struct rt_camera rt_camera; /* Camera: rays, frame, camera-relative object data */

/* ------------------------------------------------ host-side construction */

/* read_ply (TD/read_ply.cpp:13-152): mode 0 "x y z", 1 "x y z c i",
 * 2 "x y z nx ny nz".  Accepts the "end_header" header and the headerless
 * "[ply\n]nv\nnf\n" prelude (the reference hangs on those, H9).  Outputs are
 * allocated by the library; release with rt_host_free. */
int rt_read_ply(const char* path, int mode, float** points9, uint32_t* ntri,
                rt_leaf_aabb** leafs);

/* The face-assembly half of read_ply (TD/read_ply.cpp:67-149) on an indexed
 * mesh: arity[f] in {3,4}, idx = concatenated face indices. */
int rt_mesh_assemble(const float* verts, int64_t nvert, const int32_t* arity,
                     const int32_t* idx, int64_t nface, float** points9,
                     uint32_t* ntri, rt_leaf_aabb** leafs);

void rt_host_free(void* p);

/* Trixel::set_sorted_voxels + Trixel::create_kd (TD/Trixel.h:135-473,
 * TD/sort.h:11-60): the identical node array, built in parallel.
 * nodes must hold 2*ntri-1 entries.  nthreads <= 0: hardware concurrency. */
int rt_kd_build(const rt_leaf_aabb* leafs, uint32_t ntri, rt_kd_node* nodes,
                int nthreads);

/* The same build on a GPU: byte-identical nodes.  The
 * six merge sorts are stable radix sorts fed in descending position order
 * (merge_sort's tie order, TD/sort.h:25-60), each BFS level's stable
 * partitions (TD/Trixel.h:214-327) one scan and one scatter over all six
 * lists.  leafs/nodes are host arrays; the device work runs on `stream`
 * (hipStream_t or NULL) of `device` and is synchronised before returning. */
int rt_kd_build_gpu(int device, const rt_leaf_aabb* leafs, uint32_t ntri, rt_kd_node* nodes, void* stream);

/* Camera::Camera basis (TD/Camera.cpp:5-67). */
int rt_camera_basis(int32_t w, int32_t h, float f_w, float f_h, float focal,
                    const float pos[3], const float look_at[3], const float up[3],
                    rt_camera_basis_t* out);

/* WinMain's film width ((float)w/h)*.024f (TD/WinMain.cpp:29,69-70). */
float rt_film_w(int32_t w, int32_t h);

/* ----------------------------------------------------------- device path */

int rt_device_count(int* count);

/* Trixel::Trixel + init_trixels_device_memory (TD/Trixel.h:87-133,
 * TD/Trixel.cu:266-289 / init_tri_mem_cuda :11-27).  rad3 = Color::rad per
 * triangle (r,g,b floats).  Copies its inputs. */
int rt_scene_create(int device, const float* points9, const float* rad3,
                    uint32_t ntri, rt_scene** out);

/* The H2D copy at the end of Trixel::create_kd (TD/Trixel.h:380).  Validates
 * the tree (BFS order, 2*ntri-1 nodes, leaves cover every triangle once). */
int rt_scene_set_kd(rt_scene* s, const rt_kd_node* nodes, uint64_t nnode);

/* Trixel::set_sorted_voxels + create_kd + the H2D copy (TD/Trixel.h:135-473)
 * in one call, built on the scene's device (rt_kd_build_gpu) and left there:
 * no node array crosses PCIe.  Equivalent to rt_kd_build + rt_scene_set_kd. */
int rt_scene_build_kd(rt_scene* s, const rt_leaf_aabb* leafs, uint32_t ntri, void* stream);
/* Copies the scene's node array (2*ntri-1 rt_kd_node) to the host. */
int rt_scene_read_kd(rt_scene* s, rt_kd_node* nodes, uint64_t nnode);

/* Layout knobs of a scene (not in the reference; every setting renders the
 * identical frame): RT_SCENE_ORDER = the order of the dense interior records
 * the KD kernels read (0: BFS, the reference's kd_tree_node order; 1: DFS
 * preorder; 2: treelets of RT_SCENE_TREELET_HEIGHT levels, consecutive, in
 * DFS order).  Takes effect at once (cameras re-derive their records). */
#define RT_SCENE_ORDER 1
#define RT_SCENE_TREELET_HEIGHT 2
/* get only: the deepest node depth whose two children are interior records
 * at positions 2i + 1, 2i + 2 of the node's position i (BFS order: every
 * depth below floor(log2 ntri) - 1), -1 when none: the wave-cooperative
 * kernel's two-level iterations load a node's children's records in the same
 * round trip as its own up to that depth (camera debug bit 1024: off). */
#define RT_SCENE_TWO_LEVEL_DEPTH 3
int rt_scene_set_option(rt_scene* s, int32_t key, int32_t value);
int rt_scene_get_option(const rt_scene* s, int32_t key, int32_t* value);

/* Camera::Camera + init_camera_device_memory (TD/Camera.cpp:5-117,
 * TD/Camera.cu:112-136). */
int rt_camera_create(int device, int32_t w, int32_t h, float f_w, float f_h,
                     float focal, const float pos[3], const float look_at[3],
                     const float up[3], rt_camera** out);

/* Camera::add_object -> init_camera_trixel_device_memory +
 * init_camera_voxel_device_memory (TD/Camera.cpp:118-210,
 * TD/Trixel.cu:244-264, TD/Camera.cu:137-187).  The reference keeps only the
 * last object (object_list[0] colours, the second add overwrites the camera
 * buffers); so does this. */
int rt_camera_add_object(rt_camera* c, rt_scene* s);

/* One frame: bg fill -> intersect -> Phong, i.e. the steady state of
 * Object::render + Camera::color_pixels (TD/WinMain.cpp:212-237 ->
 * intersect_trixels_device TD/Trixel.cu:210-242, color_camera_device
 * TD/Camera.cu:70-87) without the D2H copy.  xform = the object's rot_m rows
 * (x.i x.j x.k x.w, y.., z..) or NULL for identity.  tile NULL = full frame.
 * stream = hipStream_t or NULL (default stream).  Writes the camera's own
 * frame buffers. */
int rt_render(rt_camera* c, const float* xform, uint32_t mode, uint32_t flags,
              const rt_tile* tile, void* stream);

/* As rt_render, into caller-owned device buffers (argb: packed pixels of the
 * tile, hit: same count of int64 or NULL). */
int rt_render_into(rt_camera* c, const float* xform, uint32_t mode, uint32_t flags,
                   const rt_tile* tile, uint32_t* d_argb, int64_t* d_hit, void* stream);

/* The frame the reference's window shows (TD/WinMain.cpp:212-237), ghosting
 * included.  The window's buffer persists: color_pixels(PHONG) overwrites
 * only the pixels whose ray hit (color_cam_cuda tests rmi >= 0,
 * TD/Camera.cu:27-61) before the blit, and color_pixels(SET) resets it to the
 * background and, through the missing `break`, this frame's Phong again
 * (TD/Camera.cu:77-84).  So the displayed frame k is the clean frame k-1
 * (background + Phong) overwritten by frame k's Phong on frame k's hits, and
 * frame 0 shows 0x00000000 where it misses (init_cam_mem_cuda zeroes the
 * buffer, TD/Camera.cu:98).  d_clean holds the previous clean frame on entry
 * (all zeros before the first frame) and this frame's on exit (what
 * rt_render_into writes); d_display receives the displayed frame.  One
 * traversal per frame; the two buffers must be distinct. */
int rt_render_display(rt_camera* c, const float* xform, uint32_t mode, uint32_t flags, const rt_tile* tile,
                      uint32_t* d_clean, uint32_t* d_display, int64_t* d_hit, void* stream);

/* Pixels in one rank's packed buffer (uniform across ranks). */
int64_t rt_tile_packed_pixels(int32_t w, int32_t h, int32_t nranks);

/* Rank 0 side of the frame gather: d_gathered = nranks packed buffers back to
 * back -> d_frame (w*h).  Runs on `stream`. */
int rt_unpack_bands(int device, int32_t w, int32_t h, int32_t nranks,
                    const uint32_t* d_gathered, uint32_t* d_frame, void* stream);

/* Multi-GPU frame gather over RCCL (the reference is
 * single-GPU, cudaSetDevice(0) at TD/Trixel.cu:213, so nothing is replaced).
 * rt_comm_unique_id on rank 0, the 128 bytes broadcast by the caller (e.g.
 * torch.distributed), then rt_comm_create on every rank (collective, like
 * ncclCommInitRank).  rt_comm_gather_frame is stream-ordered on `stream`,
 * for the frame `cam` rendered with (xform, mode) into d_local (this rank's
 * packed band buffer, rt_render_into with rt_tile{nranks, rank}): only the
 * rectangle rt_frame_rect names travels -- ranks != 0 pack their part of it
 * into d_scratch (rt_tile_packed_pixels u32) and send it to rank 0; rank 0
 * receives the peers' parts into d_scratch ((N-1) * rt_tile_packed_pixels
 * u32) and assembles d_frame (w*h) from them, its own d_local and the
 * background.  On rank 0 d_local may be d_frame itself: its bands were
 * rendered into the frame (RT_FLAG_FRAME_OUT, what rt_run_frames does) and
 * are left as they are.  Every rank must call it once per frame, with a camera of the
 * same resolution and options on every rank (message sizes are derived, not
 * exchanged; distributed.NativeFrameGather.verify checks this once).  A rank
 * with no part in the rectangle sends nothing, and rank 0 posts no receive
 * for it.  RCCL is loaded at run time (librccl.so.1, or the library the
 * environment variable RT_RCCL_LIB names, read once per process: the tests'
 * in-process shim); rt_comm_available() says whether it was found. */
#define RT_COMM_ID_BYTES 128
typedef struct rt_comm rt_comm;
int rt_comm_available(void);
int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
int rt_comm_create(int device, int32_t nranks, int32_t rank, const uint8_t id[RT_COMM_ID_BYTES], rt_comm** out);
int rt_comm_gather_frame(rt_comm* c, rt_camera* cam, const float* xform, uint32_t mode, const uint32_t* d_local,
                         uint32_t* d_scratch, uint32_t* d_frame, void* stream);
/* The frame rectangle (x0, x1, b0, b1): columns [x0, x1) of 8-row bands
 * [b0, b1).  Every pixel outside it is provably the background 0x00F08200
 * for a render of `cam` with (xform, mode) split over nranks: each rank's
 * far groups lie outside the root box's projected rectangle and are filled
 * by the fused kernel, which flags (device error 4) any that is not.  When
 * that does not hold for some rank (a transform, flat mode, options) the
 * rectangle is the whole frame; an empty rectangle is (0, 0, 0, 0). */
int rt_frame_rect(rt_camera* cam, const float* xform, uint32_t mode, int32_t nranks, int32_t rect[4]);
/* Pixels of `rank`'s part of the rectangle (its slots inside it), or -1. */
int64_t rt_rect_pixels(int32_t w, int32_t h, int32_t nranks, int32_t rank, const int32_t rect[4]);
/* rank's packed buffer -> its part of the rectangle, contiguous. */
int rt_pack_rect(int device, int32_t w, int32_t h, int32_t nranks, int32_t rank, const int32_t rect[4],
                 const uint32_t* d_local, uint32_t* d_out, void* stream);
/* Rank 0: the frame from its own packed buffer, the peers' parts (ranks
 * 1..N-1 back to back) and the background.  d_local0 == d_frame: rank 0's
 * bands are in the frame already (RT_FLAG_FRAME_OUT) and are not written. */
int rt_unpack_rect(int device, int32_t w, int32_t h, int32_t nranks, const int32_t rect[4],
                   const uint32_t* d_local0, const uint32_t* d_peers, uint32_t* d_frame, void* stream);
/* The frame rectangle without a device camera (no reference counterpart: the
 * reference is single-GPU).  rt_frame_geometry holds everything
 * rt_frame_rect derives it from: the camera basis (rt_camera_basis), the
 * root node's box minus the camera position (float subtraction, as
 * init_cam_voxel_mem_cuda does, TD/Camera.cu:142-147), whether the root is a
 * leaf, and the kernel-3 options that shape the tiling (RT_OPT_KERNEL,
 * RT_OPT_RAYS, RT_OPT_COARSE, RT_OPT_DEBUG).  rt_frame_rect_host(g, ...)
 * equals rt_frame_rect(cam, ...) whenever rt_camera_frame_geometry(cam, g)
 * filled g, so every rank (any process, no GPU needed) derives the same
 * message sizes; rt_camera_frame_geometry fails with RT_ERR_STATE when the
 * camera's scene has no KD tree (the host rectangle assumes one).  rt_pack_rect_host / rt_unpack_rect_host: rt_pack_rect /
 * rt_unpack_rect on host buffers (local0 distinct from frame). */
typedef struct rt_frame_geometry {
    int32_t w, h;
    float n_mod[3], u_mod[3], v_mod[3];
    float root_box[6];      /* x0, x1, y0, y1, z0, z1 relative to the camera */
    int32_t root_is_leaf;
    int32_t kernel, rays, coarse, debug;
} rt_frame_geometry;
int rt_camera_frame_geometry(rt_camera* cam, rt_frame_geometry* out);
int rt_frame_rect_host(const rt_frame_geometry* g, const float* xform, uint32_t mode, int32_t nranks, int32_t rect[4]);
int rt_pack_rect_host(int32_t w, int32_t h, int32_t nranks, int32_t rank, const int32_t rect[4],
                      const uint32_t* local, uint32_t* out);
int rt_unpack_rect_host(int32_t w, int32_t h, int32_t nranks, const int32_t rect[4], const uint32_t* local0,
                        const uint32_t* peers, uint32_t* frame);
int rt_comm_info(const rt_comm* c, int32_t* nranks, int32_t* rank);
void rt_comm_destroy(rt_comm* c);

/* A native frame loop (the headless replacement of WinMain's loop,
 * TD/WinMain.cpp:174-239, without the window): nframes frames of `cam` into
 * buffer set k = (*seq)++ % nbuf, each frame's render on render_stream and,
 * when comm is non-NULL, its rt_comm_gather_frame on comm_stream while the
 * next frame renders (a set is reused once its gather has read it).  With
 * event_every > 0 every event_every-th frame's render is bracketed by HIP
 * events on render_stream; *kernel_ms_avg / *kernel_ms_frames receive their
 * mean and count; *host_ms (may be NULL) the host time spent enqueueing the
 * frames.  Synchronises both streams before returning.  tile.nranks 0 (or
 * 1) renders the whole frame.  On rank 0 of comm (with a tile) frame j renders
 * straight into d_frame[k] (RT_FLAG_FRAME_OUT; d_local is unused there) and
 * the gather adds the peers' rows: the two lanes then share no events.
 * inflight (0 or 1: off) > 1 keeps that many frames in flight: frame j
 * renders on the library's render lane j % inflight (streams of the camera,
 * created once, each on a hardware queue of its own while queues are free),
 * the gather on the library's comm lane; the lanes start after the work
 * already queued on render_stream / comm_stream (no fork when nothing is
 * queued there), and every lane has drained when the call returns (it
 * synchronises them).  Frames that share a buffer set are
 * ordered (a set is rendered again once its last frame, or its gather, is
 * done), so nbuf must be a multiple of inflight whenever inflight > 1, with or
 * without comm (round 3 extended the rule to comm loops: a set is always
 * rendered by the same lane, so its frames stay ordered).  Frames are
 * independent reads of the scene; a frame's tail overlaps the next frame's
 * start, where one frame leaves most CUs idle.  Timing events then bracket
 * renders that share the GPU with another frame. */
#define RT_LOOP_MAX_BUF 8
#define RT_LOOP_MAX_LANES 4
/* inflight = RT_LOOP_MULTIFRAME: a static scene's frames (no comm, no xforms)
 * in launches of up to 128 frames, each one grid of every frame's blocks in
 * frame order (blocks are dispatched in index order), so frame j + 1's
 * heaviest tiles start on the CUs frame j's tail frees; frame j writes set
 * j % nbuf (every frame of a static scene is the same frame).  KD mode with
 * kernel 3, flags 0 and the fused far fill; otherwise (and until a cost order
 * exists) frames launch one at a time.  event_every > 0 brackets each launch;
 * *kernel_ms_avg is then their time per frame. */
#define RT_LOOP_MULTIFRAME (-1)
typedef struct rt_frame_loop {
    const float* xform;
    uint32_t mode, flags;
    rt_tile tile;
    int32_t nbuf;
    uint32_t* d_local[RT_LOOP_MAX_BUF];
    uint32_t* d_scratch[RT_LOOP_MAX_BUF];
    uint32_t* d_frame[RT_LOOP_MAX_BUF];
    void* render_stream;
    void* comm_stream;
    int32_t event_every;
    int32_t inflight;
    /* nxforms > 0: frame k = (*seq) of the loop renders with the object
     * transform xforms + 12 * (k % nxforms) (a moving object's poses, one per
     * frame, e.g. Object::transform after each input tick), instead of xform */
    const float* xforms;
    int32_t nxforms;
} rt_frame_loop;
int rt_run_frames(rt_camera* cam, rt_comm* comm, const rt_frame_loop* loop, int32_t nframes, int64_t* seq,
                  double* kernel_ms_avg, int32_t* kernel_ms_frames, double* host_ms);

/* The D2H copy of color_camera_device (TD/Camera.cu:84) and d_rmi.index.
 * Synchronises the device.  argb: w*h u32 0x00RRGGBB; hit may be NULL. */
int rt_read_frame(rt_camera* c, uint32_t* argb, int64_t* hit);

/* Frame delivery: the reference copies every frame
 * to the host synchronously (cudaMemcpy in color_camera_device,
 * TD/Camera.cu:84; blit in TD/WinMain.cpp:217).  These let a frame loop copy
 * frame k to pinned host memory on a copy stream while frame k+1 renders.
 * rt_pinned_alloc / rt_pinned_free: page-locked host memory (hipHostMalloc).
 * rt_frame_copy_async: npix u32 from device d_argb to host h_argb, ordered
 * on `stream` (a hipStream_t or NULL); no synchronisation. */
int rt_pinned_alloc(size_t bytes, void** out);
void rt_pinned_free(void* p);
int rt_frame_copy_async(int device, const uint32_t* d_argb, uint32_t* h_argb, int64_t npix, void* stream);

/* Counters accumulated by RT_FLAG_COUNT renders: [0] interior visits,
 * [1] leaf visits, [2] accepted hits, [3] hit pixels, [4] interior visits
 * that descended.  reset != 0 zeroes them after reading.  Synchronises. */
int rt_camera_counters(rt_camera* c, uint64_t out[5], int reset);

/* The camera's device error word, which every render ORs into: 1 = DFS
 * stack overflow (kernels 1-2), 2 = item pool overflow (kernel 3), 4 = a
 * fused far group that was not provably background (kernel 3; the gathered
 * frame's background then is not the rendered one), 8 = a tile-order entry
 * outside the fine grid (kernel 3; that block is skipped).  The reference has no
 * equivalent (its status is the last sync, TD/Trixel.cu:227-240).
 * Synchronises the device; *err receives the word; reset != 0 clears it.
 * Returns RT_OK even when *err is non-zero (the word is the report). */
int rt_camera_error(rt_camera* c, int32_t* err, int reset);

/* Kernel launch geometry and the traversal stack depth in use. */
int rt_camera_info(const rt_camera* c, int32_t* w, int32_t* h, int32_t* max_depth);

/* Tuning knobs (not in the reference): key 1 = KD kernel (2: per-lane DFS
 * in the reference's visiting order, child-box records, its counters are the
 * reference's; 3: wave-cooperative item pool, default), key 2 = tile dispatch order (0: XCD-
 * contiguous, 1: natural, 2: centre-out, 3: heaviest first by the cost an
 * earlier frame measured, default; every 16th frame of kernel 3 writes
 * its units' costs into page-locked host memory, read once that frame's
 * event has completed; no samples while the stream is captured; 4: per XCD
 * (block b on XCD b % 8) over 8 Morton runs of equal cost, heaviest first in
 * each; 5: per XCD over 8 row bands of equal tile count, heaviest first in
 * each -- orders 0, 4 and 5 pad multi-frame launches to 8 blocks per frame).
 * Every setting renders the identical frame. */
#define RT_OPT_KERNEL 1
#define RT_OPT_TILE_ORDER 2
#define RT_OPT_RAYS 3 /* kernel 3: pixels per wave (32, 16, 8; 0 = auto, default: 8 when this rank's
                         share of the object's screen rectangle is too small to fill the GPU with 16,
                         else 16; inside rt_run_frames' multi-frame launches (RT_LOOP_MULTIFRAME) 32
                         when that rectangle holds fewer than 8,192 16-pixel units, else 16) */
#define RT_OPT_ITEMS 4 /* kernel 3: items each lane pops per iteration (1, 2 default; 65..128: two only when the pool holds at least that many) */
#define RT_OPT_COARSE 5 /* kernel 3: 8x8 groups per wave outside the root box's screen rectangle (0..32, 8 default, 0 = off) */
/* kernel 3, shadow rays: the order the any-hit walk pushes children in (0..3;
 * -1 = timed, default: every 2048 shadow frames each order runs 3 frames
 * bracketed by events and the fastest is kept; never blocks, skipped under
 * stream capture).  Get returns the order in use. */
#define RT_OPT_SHADOW_ORDER 6
/* Flat-list kernel form (same frame): 9 = one pass over the signed pair
 * layout, packed float2 arithmetic, v's numerator first (a wave whose rays
 * all have V <= 0 skips the rest of the pair), the next pair's scalar loads
 * in flight during a pair's tests; 12 (default) = 9 over 16 chunks of the
 * list (a grid of short waves; the chunks' nearest hits meet in a per-pixel
 * 64-bit minimum, then a shading pass; counting renders take 9). */
#define RT_OPT_FLAT 7
#define RT_OPT_RAYS_USED 8 /* get only: the pixels per wave the last kernel-3 render used */
/* get only: tiles of the current cost order (tile order 3, 16- and 8-ray
 * units) rendered as two halves (a 16-ray unit as two 8-ray rows, an 8-ray
 * unit as two 4-pixel halves): those costlier than 50 % of the heaviest tile
 * in grids of fewer than 2,048 tiles and 75 % in larger ones, at most a
 * quarter of the tiles.  Costs are pool iterations per unit (8 slots per
 * tile: the 4 units and the second halves).  The frame is the same either
 * way. */
#define RT_OPT_SPLIT_USED 9
/* Keys 10 and 11 are retired (ABI 2): RT_OPT_COOP_USED and
 * RT_OPT_FRAME_GROUP of round 4; both are rejected. */
/* get only: which walks of the last kernel-3 render took the exact
 * single-precision slab and ordering forms (the frame is the same either
 * way): bit 0 the nearest-hit walk (its frame proved the float entry test),
 * bit 1 the shadow walk (the light proved it), bit 2 the walk ran under an
 * object transform; 0 when neither proof held */
#define RT_OPT_FAST_USED 12
/* get only: how many times this camera restarted a tiling from the cost
 * order it last measured there (a camera alternating between two tilings,
 * e.g. rt_run_frames' multi-frame 32-ray rule and the per-frame 16-ray one) */
#define RT_OPT_ORDER_RESTORES 13
/* get only: the fine tiles (one kRays-pixel unit per wave) of the last
 * kernel-3 render; every other 8x8 group was a coarse or far group */
#define RT_OPT_FINE_TILES 14
int rt_camera_set_option(rt_camera* c, int32_t key, int32_t value);
int rt_camera_get_option(const rt_camera* c, int32_t key, int32_t* value);

/* Diagnostics (key 100 of rt_camera_set_option: 1 = skip traversal,
 * 2 = per-wave (start clock, end clock, max visits) records, 16 = counted
 * shadow walks stop at occluders like timed ones): copies up to
 * n u64 of the record buffer; returns the count or a negative status. */
#define RT_OPT_DEBUG 100
#define RT_OPT_POOL_CAP 101 /* tests: shrink the wave-cooperative kernel's item pool (89..640) */
int64_t rt_camera_debug_read(rt_camera* c, uint64_t* out, int64_t n);

/* Object motion: the reference's keyboard transform
 * path, driven headlessly.  An rt_object is Object's motion state (its
 * Quaternion, host rot_m, device d_rot_m, init_face/cur_face; TD/Object.h,
 * TD/Camera.cpp:131-134).  rt_object_transform replaces Object::transform ->
 * transform_camera_voxel_device_memory (TD/Object.cpp:14-17,
 * TD/Camera.cu:254-335) with the reference's selector values
 * (TD/platform_common.h:15-20); an unknown selector is RT_ERR_INVALID (the
 * reference ignores it).  rt_object_tick applies one input tick's held keys
 * in the order of TD/WinMain.cpp:186-209 (R, W, S, Q, E, T).
 * rt_object_xform gives the device rot_m rows that rt_render's xform takes
 * (what intersect_voxel_cuda reads, TD/Trixel.cu:60-66). */
typedef struct rt_object rt_object;
#define RT_TRANSLATE_XYZ 30
#define RT_TRANSLATE_X 31
#define RT_TRANSLATE_Z 32
#define RT_ROTATE_PY 10
#define RT_ROTATE_NY 11
#define RT_KEY_R 1u   /* rotate +y: t_vec (0, 0.0995, 0, 0.995)  */
#define RT_KEY_W 2u   /* forward:   (n, +speed), TRANSLATE_Z      */
#define RT_KEY_S 4u   /* back:      (n, -speed)                   */
#define RT_KEY_Q 8u   /* strafe:    (u, +speed), TRANSLATE_X      */
#define RT_KEY_E 16u  /* strafe:    (u, -speed)                   */
#define RT_KEY_T 32u  /* rotate -y: (0, -0.0995, 0, 0.995)        */
#define RT_KEYS_ALL 63u
/* cam_pos, cam_n, cam_u: the camera's o_prop.pos/n/u (rt_camera_basis);
 * cam_speed: 0.005 in the reference (TD/WinMain.cpp:170). */
int rt_object_create(const float cam_pos[3], const float cam_n[3], const float cam_u[3], float cam_speed,
                     rt_object** out);
int rt_object_transform(rt_object* o, const float t_vec[4], int32_t select);
int rt_object_tick(rt_object* o, uint32_t held_keys);
int rt_object_xform(const rt_object* o, float xform[12]);
/* Host-side state for tests (any pointer may be NULL): quaternion (i j k w),
 * host rot_m rows, init_face, cur_face. */
int rt_object_state(const rt_object* o, float quat[4], float host_rot[12], float init_face[4], float cur_face[4]);
void rt_object_destroy(rt_object* o);

void rt_scene_destroy(rt_scene* s);
void rt_camera_destroy(rt_camera* c);

const char* rt_last_error_string(void);
int rt_abi_version(void);
/* Build provenance: the SHA-256 (hex) of the sources (csrc/, include/) and the
 * compile/link flags this library was built from (cpp_cuda_raytracer_dev_amd/
 * build.py source_id); the Python binding refuses a library whose id differs
 * from the tree's. */
const char* rt_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_MI355X_H */
