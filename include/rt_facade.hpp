// rt_facade.hpp -- the reference's host-side C++ construction API, header-only,
// layered on the C ABI of rt_mi355x.h.  Same class and function names, the
// same argument meaning, status codes instead of cudaError_t (0 = success):
//
//   read_ply            TD/read_ply.cpp:13        -> rt_read_ply
//   Trixel              TD/Trixel.h:39-478        -> rt_scene_*, rt_kd_build
//   Camera              TD/Camera.h:15-97         -> rt_camera_*
//   Object              TD/Object.h:10-19         -> rt_object_* (motion)
//   Quaternion          TD/Quaternion.h:5-24      (the rot_m the kernel reads)
//   Input               TD/Input.h:3-15           (t_vec of a transform)
//   Color               TD/Color.h:4-14
//
// The frame is the steady state of the reference's loop (TD/WinMain.cpp:
// 212-237): Object::render runs the fused bg-fill -> intersect -> Phong
// kernel; Camera::color_pixels copies it to h_mem.h_color.c (the D2H of
// TD/Camera.cu:84).  Win32 is out of scope: the keyboard
// loop's transforms are Object::transform / Object::key_tick (rt_object_*),
// and Object::set_transform takes a ready rot_m.
#pragma once

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rt_mi355x.h"

namespace rtmi {

typedef float T_fp;        // TD/typedefs.h:15 (PPP_TAG == 0)
typedef uint32_t T_uint;
typedef int32_t s32;
typedef int64_t s64;
typedef uint8_t u8;
typedef uint32_t u32;

constexpr u8 SET_COLOR_TAG = 1;     // TD/Camera.h:13
constexpr u8 PHONG_COLOR_TAG = 2;   // TD/Camera.h:14
constexpr u8 TRIXEL_OBJECT_TAG = 0; // TD/Object.h:3
constexpr u8 TRANSLATE_XYZ = RT_TRANSLATE_XYZ;  // TD/platform_common.h:15-20
constexpr u8 TRANSLATE_X = RT_TRANSLATE_X;
constexpr u8 TRANSLATE_Z = RT_TRANSLATE_Z;
constexpr u8 ROTATE_TRI_PY = RT_ROTATE_PY;
constexpr u8 ROTATE_TRI_NY = RT_ROTATE_NY;
constexpr u32 RENDER_MODE_KD = RT_MODE_KD;
constexpr u32 RENDER_MODE_FLAT = RT_MODE_FLAT;

typedef rt_leaf_aabb kd_leaf_sort;  // the AABB half of kd_leaf_sort (TD/Trixel.h:20-30)
struct kd_vertex { T_fp x, y, z; }; // TD/Trixel.h:17

// TD/read_ply.cpp:13.  The reference frees the vertex list before returning;
// here *vertex_list is set to null and *num_vert to 0 likewise.  Release
// *points_list and *kd_leafs with rt_host_free.  Returns an rt_status.
inline int read_ply(const char* file_name, T_fp** points_list, T_uint* num_tri, kd_leaf_sort** kd_leafs,
                    kd_vertex** vertex_list, T_uint* num_vert, u8 mode) {
    if (vertex_list) *vertex_list = nullptr;
    if (num_vert) *num_vert = 0;
    return rt_read_ply(file_name, mode, points_list, num_tri, kd_leafs);
}

// TD/Color.h:4-14: per-triangle radiance (the u32 colours are unused by the path).
class Color {
public:
    struct radiance { T_fp r, g, b; };
    u32* c = nullptr;
    radiance* rad = nullptr;
};

// TD/Quaternion.h: rot_m rows x, y, z as (i, j, k, w); identity at construction.
class Quaternion {
public:
    T_fp rot_m[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
};

// TD/Input.h:3-15 without the Win32 buttons: set_quat stores the four floats
// as the transform vector t_vec (TD/Input.cpp:16-19).
class Input {
public:
    T_fp t_vec[4] = {0, 0, 0, 0};
    void set_vec(T_fp x, T_fp y, T_fp z, T_fp w) { t_vec[0] = x; t_vec[1] = y; t_vec[2] = z; t_vec[3] = w; }
    void set_quat(T_fp x, T_fp y, T_fp z, T_fp w) { set_vec(x, y, z, w); }
};

class Camera;

class Trixel {
public:
    u8 object_tag = TRIXEL_OBJECT_TAG;
    s64 num_trixels = 0;
    s64 num_voxels = 0;
    int device = 0;
    int status = RT_OK;  // status of the constructor (the reference prints and continues)

    // Trixel(s64, T_fp*, Color*) (TD/Trixel.h:87-133) + init_trixels_device_memory
    Trixel(s64 num_t, T_fp* points_data, Color* color_data, int dev = 0) : num_trixels(num_t), device(dev) {
        num_voxels = num_t * 2 - 1;
        std::vector<float> rad((size_t)num_t * 3);
        for (s64 i = 0; i < num_t; i++) {
            rad[3 * i] = color_data->rad[i].r;
            rad[3 * i + 1] = color_data->rad[i].g;
            rad[3 * i + 2] = color_data->rad[i].b;
        }
        status = rt_scene_create(device, points_data, rad.data(), (uint32_t)num_t, &scene_);
    }
    ~Trixel() { rt_scene_destroy(scene_); }
    Trixel(const Trixel&) = delete;
    Trixel& operator=(const Trixel&) = delete;

    // TD/Trixel.h:386-473: keeps a copy of the leaf AABBs for create_kd.
    int set_sorted_voxels(kd_leaf_sort* voxel_list, T_uint num_leaf_voxels) {
        if (num_leaf_voxels == 0) return 0;
        leafs_.assign(voxel_list, voxel_list + num_leaf_voxels);
        return 0;
    }

    // TD/Trixel.h:135-385: -12 if set_sorted_voxels was not called.
    int create_kd(int nthreads = 0) {
        if (leafs_.empty()) return -12;
        std::vector<rt_kd_node> nodes((size_t)(2 * leafs_.size() - 1));
        int rc = rt_kd_build(leafs_.data(), (uint32_t)leafs_.size(), nodes.data(), nthreads);
        if (rc == RT_OK) rc = rt_scene_set_kd(scene_, nodes.data(), nodes.size());
        leafs_.clear();
        leafs_.shrink_to_fit();
        return rc;
    }

    // TD/Trixel.h:474-476 (m selects KD or flat here; the reference ignores it)
    inline int intersect_trixels(Camera* c, Quaternion* q, u32 m = RENDER_MODE_KD);

    rt_scene* handle() const { return scene_; }

private:
    rt_scene* scene_ = nullptr;
    std::vector<kd_leaf_sort> leafs_;
};

class Object {
public:
    Trixel* trixel_list = nullptr;
    Quaternion* quat = nullptr;

    explicit Object(Trixel* x) : trixel_list(x), quat(&own_) {}
    Object(Trixel* x, Quaternion* q) : trixel_list(x), quat(&own_), own_(*q) {}
    ~Object() { rt_object_destroy(motion_); }
    Object(const Object&) = delete;
    Object& operator=(const Object&) = delete;
    u8 getTag() const { return trixel_list->object_tag; }
    // Object::render (TD/Object.cpp:10-12)
    int render(Camera* c, u32 mode = RENDER_MODE_KD) { return trixel_list->intersect_trixels(c, quat, mode); }
    // Object::transform (TD/Object.cpp:14-17): needs Camera::add_object first
    int transform(Input* dq, u8 transform_select) {
        if (!motion_) return RT_ERR_STATE;
        int rc = rt_object_transform(motion_, dq->t_vec, transform_select);
        return rc ? rc : rt_object_xform(motion_, own_.rot_m);
    }
    // one tick of TD/WinMain.cpp:186-209 with RT_KEY_* held
    int key_tick(uint32_t held_keys) {
        if (!motion_) return RT_ERR_STATE;
        int rc = rt_object_tick(motion_, held_keys);
        return rc ? rc : rt_object_xform(motion_, own_.rot_m);
    }
    // replaces the transform state with a ready matrix
    void set_transform(const T_fp rot_m[12]) { memcpy(own_.rot_m, rot_m, sizeof own_.rot_m); }
    // Camera::add_object's init_face / cur_face / quat copy (TD/Camera.cpp:131-134)
    int attach_motion(const float pos[3], const float n[3], const float u[3], T_fp cam_speed) {
        rt_object_destroy(motion_);
        motion_ = nullptr;
        int rc = rt_object_create(pos, n, u, cam_speed, &motion_);
        return rc ? rc : rt_object_xform(motion_, own_.rot_m);
    }

private:
    Quaternion own_;
    rt_object* motion_ = nullptr;
};

class Camera {
public:
    struct film_properties {
        struct resolution { u32 w, h; uint64_t count; } res;
    } f_prop{};
    struct pixel_memory {
        struct { u32* c = nullptr; } h_color;      // the frame, 0x00RRGGBB, row 0 = bottom
        struct { s64* index = nullptr; } h_rmi;    // hit triangle per pixel (-1 miss)
    } h_mem;
    int status = RT_OK;

    // Camera(...) (TD/Camera.h:86-91, TD/Camera.cpp:5-117)
    Camera(s32 r_w, s32 r_h, T_fp f_w, T_fp f_h, T_fp fclen, T_fp p_x, T_fp p_y, T_fp p_z, T_fp la_x, T_fp la_y,
           T_fp la_z, T_fp up_x, T_fp up_y, T_fp up_z, int dev = 0) {
        f_prop.res.w = (u32)r_w;
        f_prop.res.h = (u32)r_h;
        f_prop.res.count = (uint64_t)r_w * (uint64_t)r_h;
        const float pos[3] = {p_x, p_y, p_z}, la[3] = {la_x, la_y, la_z}, up[3] = {up_x, up_y, up_z};
        status = rt_camera_create(dev, r_w, r_h, f_w, f_h, fclen, pos, la, up, &cam_);
        memcpy(pos_, pos, sizeof pos_);
        rt_camera_basis_t b;
        if (status == RT_OK) status = rt_camera_basis(r_w, r_h, f_w, f_h, fclen, pos, la, up, &b);
        if (status == RT_OK) {
            memcpy(n_, b.n, sizeof n_);
            memcpy(u_, b.u, sizeof u_);
        }
        color_.assign(f_prop.res.count, 0u);
        rmi_.assign(f_prop.res.count, -1);
        h_mem.h_color.c = color_.data();
        h_mem.h_rmi.index = rmi_.data();
    }
    ~Camera() { rt_camera_destroy(cam_); }
    Camera(const Camera&) = delete;
    Camera& operator=(const Camera&) = delete;

    // Camera::add_object (TD/Camera.cpp:118-142)
    int add_object(Object* new_object) {
        if (new_object->getTag() != TRIXEL_OBJECT_TAG) return 0;
        objects_.push_back(new_object);
        int rc = new_object->attach_motion(pos_, n_, u_, cam_speed);
        return rc ? rc : rt_camera_add_object(cam_, new_object->trixel_list->handle());
    }

    // Camera::color_pixels (TD/Camera.cpp:229): the frame to h_mem.h_color.c
    // (and the hit buffer when the last render wrote one).
    int color_pixels(u8 color_tag_select = PHONG_COLOR_TAG) {
        (void)color_tag_select;  // both tags show the steady-state frame
        return rt_read_frame(cam_, h_mem.h_color.c, write_hit_ ? h_mem.h_rmi.index : nullptr);
    }

    int render_with(const Quaternion* q, u32 mode) {
        return rt_render(cam_, q ? q->rot_m : nullptr, mode, write_hit_ ? RT_FLAG_WRITE_HIT : 0u, nullptr, nullptr);
    }
    void keep_hit_buffer(bool on) { write_hit_ = on; }
    rt_camera* handle() const { return cam_; }
    T_fp cam_speed = .005f;  // TD/WinMain.cpp:170

private:
    rt_camera* cam_ = nullptr;
    float pos_[3] = {0, 0, 0}, n_[3] = {0, 0, 1}, u_[3] = {1, 0, 0};
    std::vector<u32> color_;
    std::vector<s64> rmi_;
    std::vector<Object*> objects_;
    bool write_hit_ = false;
};

inline int Trixel::intersect_trixels(Camera* c, Quaternion* q, u32 m) { return c->render_with(q, m); }

// WinMain's film width ((float)w / h) * .024f (TD/WinMain.cpp:29,69-70).
inline T_fp film_w(s32 w, s32 h) { return rt_film_w(w, h); }

}  // namespace rtmi
