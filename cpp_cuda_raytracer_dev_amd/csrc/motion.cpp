// Object motion: the reference's keyboard transform path, driven headlessly
// (SURVEY.md §8f rank 3).  TD/ = TEST_Dungeonrun/ in the reference.
//
// Per key the reference updates the object's quaternion and its host rot_m
// (TD/vector.cpp:38-65, TD/Camera.cu:254-335) and, through two 1-thread
// kernels, the device rot_m the hot kernel reads (TD/Trixel.cu:60-66):
//   * update_voxel_transform_m_translate_cuda (TD/Camera.cu:188-192) adds
//     scale * t.x * t.d to the device translation column.  nvcc contracts that
//     into fma(scale * t.x, t.d, w) (FMA contraction is on in the reference's
//     build), while the host line `w += t.d * t.x` rounds the
//     product first, so host and device columns can drift apart by an ulp per
//     translate;
//   * set_rotation_matrix (TD/Quaternion.cu:4-10) copies the host rows to the
//     device on every rotate, which resynchronises them.
// Both copies are kept here; rt_object_xform returns the device one.  The
// translate kernel translate_cam_voxel_mem_cuda (TD/Camera.cu:227-252) is
// never launched by the reference (status_lauch_and_sync only checks errors,
// TD/vector.cuh:15-18), so camera-relative records are not touched.
//
// Host float arithmetic follows MSVC x64 /fp:precise: IEEE single, no
// contraction (this file is built with -ffp-contract=off and x86-64 has no
// FMA in the baseline ISA).  vector_norm's union reads 8 bytes of which 4 are
// written (TD/vector.cpp:13-26); like the camera setup (scene_host.cpp) the
// upper 4 are taken as zero.
#include <cmath>
#include <cstring>
#include <new>

#include "rt_internal.h"

using rt::fail;

namespace {

float vector_norm(float s) {  // TD/vector.cpp:13-26
    const float half = 0.5f * s;
    union { float f; uint32_t i; } u;
    u.f = half;
    u.i = 0x5f375a86u - (u.i >> 1);
    for (int k = 0; k < 8; k++) u.f = u.f * (1.5f - half * u.f * u.f);
    return u.f;
}

struct Vec4 {  // VEC4<T_fp>: x y z w, with i j k / d aliases (TD/Vector.h:45-66)
    float x, y, z, w;
    void sub(const Vec4& r) {  // operator-=, TD/Vector.h:89-94
        x = (x * w) - (r.x * r.w);
        y = (y * w) - (r.y * r.w);
        z = (z * w) - (r.z * r.w);
        w = 1.0f;
    }
    void add(const Vec4& r) {  // operator+=, TD/Vector.h:95-100
        x = (x * w) + (r.x * r.w);
        y = (y * w) + (r.y * r.w);
        z = (z * w) + (r.z * r.w);
        w = 1.0f;
    }
    void negate() { x = -x; y = -y; z = -z; }  // TD/Vector.h:105
    void normalize() {                          // normalize_Vector(VEC4*), TD/Vector.h:116-124
        float s = x * x + y * y + z * z;
        s = vector_norm(s);
        x *= s; y *= s; z *= s;
        w = 1 / s;
    }
};

}  // namespace

struct rt_object {
    Vec4 quat;        // Quaternion::vec (i j k w)
    Vec4 rot[3];      // host rot_m rows x y z (i j k w)
    Vec4 drot[3];     // device d_rot_m rows
    Vec4 init_face, cur_face;
    float cam_n[3], cam_u[3];
    float speed;
};

namespace {

// VEC4::rotate (TD/vector.cpp:38-65): an optional quaternion product
// cur_vec * new_vec that rewrites rot_m's 3x3 part, then v = rot_m * (v * reverse).
void rotate(Vec4& v, rt_object* o, const Vec4* nv, int reverse) {
    Vec4& q = o->quat;
    Vec4* R = o->rot;
    if (nv) {
        const float ti = q.x, tj = q.y, tk = q.z, tw = q.w;
        q.x = tj * nv->z - tk * nv->y + ti * nv->w + tw * nv->x;
        q.y = tk * nv->x - ti * nv->z + tj * nv->w + tw * nv->y;
        q.z = ti * nv->y - tj * nv->x + tk * nv->w + tw * nv->z;
        q.w = tw * nv->w - ti * nv->x - tj * nv->y - tk * nv->z;
        R[0].x = (1 - 2 * q.y * q.y - 2 * q.z * q.z);
        R[0].y = (2 * q.x * q.y - 2 * q.z * q.w);
        R[0].z = (2 * q.x * q.z + 2 * q.y * q.w);
        R[1].x = (2 * q.x * q.y + 2 * q.z * q.w);
        R[1].y = (1 - 2 * q.x * q.x - 2 * q.z * q.z);
        R[1].z = (2 * q.y * q.z - 2 * q.x * q.w);
        R[2].x = (2 * q.x * q.z - 2 * q.y * q.w);
        R[2].y = (2 * q.y * q.z + 2 * q.x * q.w);
        R[2].z = (1 - 2 * q.x * q.x - 2 * q.y * q.y);
    }
    const float fr = (float)reverse;
    const float tx = v.x * fr, ty = v.y * fr, tz = v.z * fr;
    v.x = (tx * R[0].x + ty * R[0].y + tz * R[0].z);
    v.y = (tx * R[1].x + ty * R[1].y + tz * R[1].z);
    v.z = (tx * R[2].x + ty * R[2].y + tz * R[2].z);
}

// update_voxel_transform_m_translate_cuda (TD/Camera.cu:188-192), contracted
void device_translate(rt_object* o, const Vec4& t, int scale) {
    const float fs = (float)scale;
    o->drot[0].w = std::fmaf(fs * t.x, t.w, o->drot[0].w);
    o->drot[1].w = std::fmaf(fs * t.y, t.w, o->drot[1].w);
    o->drot[2].w = std::fmaf(fs * t.z, t.w, o->drot[2].w);
}

}  // namespace

extern "C" int rt_object_create(const float cam_pos[3], const float cam_n[3], const float cam_u[3], float cam_speed,
                                rt_object** out) {
    if (!cam_pos || !cam_n || !cam_u || !out) return fail(RT_ERR_INVALID, "rt_object_create: null argument");
    *out = nullptr;
    rt_object* o = new (std::nothrow) rt_object;
    if (!o) return fail(RT_ERR_NOMEM, "rt_object_create: out of memory");
    o->quat = Vec4{0, 0, 0, 1};                      // Quaternion(3), TD/Quaternion.cpp:17-22
    for (int r = 0; r < 3; r++) {
        o->rot[r] = Vec4{r == 0 ? 1.0f : 0.0f, r == 1 ? 1.0f : 0.0f, r == 2 ? 1.0f : 0.0f, 0.0f};
        o->drot[r] = o->rot[r];                      // initialize_CUDA copies the rows
    }
    o->init_face = Vec4{-cam_pos[0], -cam_pos[1], -cam_pos[2], 1.0f};  // TD/Camera.cpp:131-132
    o->cur_face = o->init_face;
    std::memcpy(o->cam_n, cam_n, sizeof(o->cam_n));
    std::memcpy(o->cam_u, cam_u, sizeof(o->cam_u));
    o->speed = cam_speed;
    *out = o;
    return RT_OK;
}

extern "C" int rt_object_transform(rt_object* o, const float t_vec[4], int32_t select) {
    if (!o || !t_vec) return fail(RT_ERR_INVALID, "rt_object_transform: null argument");
    Vec4 tv{t_vec[0], t_vec[1], t_vec[2], t_vec[3]};
    switch (select) {
    case RT_TRANSLATE_XYZ:
    case RT_TRANSLATE_X:
    case RT_TRANSLATE_Z:  // TD/Camera.cu:258-287
        o->init_face.sub(tv);
        rotate(tv, o, nullptr, -1);
        o->rot[0].w += tv.w * tv.x;
        o->rot[1].w += tv.w * tv.y;
        o->rot[2].w += tv.w * tv.z;
        device_translate(o, tv, 1);
        o->init_face.normalize();
        o->cur_face = o->init_face;
        rotate(o->cur_face, o, nullptr, -1);
        o->cur_face.negate();
        return RT_OK;
    case RT_ROTATE_PY:
    case RT_ROTATE_NY: {  // TD/Camera.cu:288-330
        Vec4 t = o->init_face;
        rotate(t, o, &tv, -1);
        for (int r = 0; r < 3; r++) o->drot[r] = o->rot[r];  // set_device_rotation
        t.add(o->cur_face);
        o->rot[0].w -= t.x * t.w;
        o->rot[1].w -= t.y * t.w;
        o->rot[2].w -= t.z * t.w;
        device_translate(o, t, -1);
        t.sub(o->cur_face);
        o->cur_face = t;
        o->cur_face.normalize();
        o->cur_face.negate();
        return RT_OK;
    }
    default:
        return fail(RT_ERR_INVALID, "rt_object_transform: unknown transform %d", (int)select);
    }
}

extern "C" int rt_object_tick(rt_object* o, uint32_t held_keys) {
    if (!o) return fail(RT_ERR_INVALID, "rt_object_tick: null object");
    if (held_keys & ~(uint32_t)RT_KEYS_ALL) return fail(RT_ERR_INVALID, "rt_object_tick: unknown key bits 0x%x", held_keys);
    // TD/WinMain.cpp:186-209, in its order; set_quat stores the 4 floats as
    // t_vec (TD/Input.cpp:16-19)
    const float kRot = (float)0.09950371902099893, kRotW = (float)0.9950371902099893;
    const float* n = o->cam_n;
    const float* u = o->cam_u;
    int rc = RT_OK;
    if (held_keys & RT_KEY_R) {
        const float t[4] = {0.0f, kRot, 0.0f, kRotW};
        if ((rc = rt_object_transform(o, t, RT_ROTATE_PY))) return rc;
    }
    if (held_keys & RT_KEY_W) {
        const float t[4] = {n[0], n[1], n[2], o->speed};
        if ((rc = rt_object_transform(o, t, RT_TRANSLATE_Z))) return rc;
    }
    if (held_keys & RT_KEY_S) {
        const float t[4] = {n[0], n[1], n[2], -o->speed};
        if ((rc = rt_object_transform(o, t, RT_TRANSLATE_Z))) return rc;
    }
    if (held_keys & RT_KEY_Q) {
        const float t[4] = {u[0], u[1], u[2], o->speed};
        if ((rc = rt_object_transform(o, t, RT_TRANSLATE_X))) return rc;
    }
    if (held_keys & RT_KEY_E) {
        const float t[4] = {u[0], u[1], u[2], -o->speed};
        if ((rc = rt_object_transform(o, t, RT_TRANSLATE_X))) return rc;
    }
    if (held_keys & RT_KEY_T) {
        const float t[4] = {0.0f, -kRot, 0.0f, kRotW};
        if ((rc = rt_object_transform(o, t, RT_ROTATE_NY))) return rc;
    }
    return RT_OK;
}

extern "C" int rt_object_xform(const rt_object* o, float xform[12]) {
    if (!o || !xform) return fail(RT_ERR_INVALID, "rt_object_xform: null argument");
    for (int r = 0; r < 3; r++) {
        xform[4 * r + 0] = o->drot[r].x;
        xform[4 * r + 1] = o->drot[r].y;
        xform[4 * r + 2] = o->drot[r].z;
        xform[4 * r + 3] = o->drot[r].w;
    }
    return RT_OK;
}

extern "C" int rt_object_state(const rt_object* o, float quat[4], float host_rot[12], float init_face[4],
                               float cur_face[4]) {
    if (!o) return fail(RT_ERR_INVALID, "rt_object_state: null object");
    auto put = [](float* d, const Vec4& v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w; };
    if (quat) put(quat, o->quat);
    if (host_rot)
        for (int r = 0; r < 3; r++) put(host_rot + 4 * r, o->rot[r]);
    if (init_face) put(init_face, o->init_face);
    if (cur_face) put(cur_face, o->cur_face);
    return RT_OK;
}

extern "C" void rt_object_destroy(rt_object* o) { delete o; }
