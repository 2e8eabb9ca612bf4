// rt_predicates.h -- the reference's double-promoted epsilon compares, and
// exact single-precision forms of them for the traversal's hot loop.
//
// The reference evaluates its epsilon tests in double (the 1e-16 literals of
// TD/vector.cuh:10-11 promote the float operands): the slab entry test
// `mint1 >= maxt0 - 1e-16 && maxt0 > -1e-16` (TD/Trixel.cu:146) and the child
// ordering `maxt0 < s2 + 1e-16`, `mint1 > s2 - 1e-16`, `s1 + 1e-16`
// (TD/Trixel.cu:150-161).  For a float x with |x| >= 2^-20 the float spacing
// around x (>= 2^-43) dwarfs 1e-16, so x -/+ 1e-16 rounded to double lies in
// (pred(x), x] / [x, succ(x)) and each test reduces to a float compare with
// one of its edge cases (equality) decided by the double form.  Tiny, NaN and
// equal operands take the double form itself.  tests/test_predicates.py
// checks every fast form against its double form on CPU (edge sets plus
// random sweeps over all binades).  These per-predicate forms (with their
// equality branches) serve the translated walks only with
// -DRT_FAST_PREDICATES: on gfx950 their branches cost more than the double
// arithmetic they skip (0.126 vs 0.118 ms per 1080p dragon frame, round 1).
// The default kernels instead take branch-free float forms wherever a frame
// PROVES that no operand is tiny (rt_kernels_impl.h kFast walks, rt_api.cpp
// fast_proof: every box's maxt0 >= 2^-20, so the entry test is the float
// mint1 >= maxt0, and the ordering compares use the exact float thresholds
// k_cam_nodes stores), and the double forms below (the *_ref functions)
// everywhere else.
#pragma once

#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD static inline
#endif

namespace rt {
namespace pred {

constexpr double kEps = 1e-16;
constexpr float kSmall = 0x1p-20f;

// Smallest float >= 1e-16 (1e-16 is not a float): (double)x > -1e-16 <=> x > -kEpsF.
RT_HD float eps_f() {
    union { uint32_t u; float f; } c = {0x24e69595u};
    return c.f;
}

// TD/Trixel.cu:146: descend into a node whose box the ray enters.
RT_HD bool enter_ref(float maxt0, float mint1) { return (double)mint1 >= (double)maxt0 - kEps && (double)maxt0 > -kEps; }
RT_HD bool enter(float maxt0, float mint1) {
#ifndef RT_FAST_PREDICATES
    return enter_ref(maxt0, mint1);
#endif
    if (maxt0 >= kSmall) return mint1 >= maxt0;
    if (maxt0 <= -kSmall) return false;
    return enter_ref(maxt0, mint1);
}

// (double)a < (double)s + 1e-16 (TD/Trixel.cu:155).
RT_HD bool lt_eps_ref(float a, float s) { return (double)a < (double)s + kEps; }
RT_HD bool lt_eps(float a, float s) {
#ifndef RT_FAST_PREDICATES
    return lt_eps_ref(a, s);
#endif
    if (a != s && fabsf(s) >= kSmall) return a < s;
    return lt_eps_ref(a, s);
}

// (double)a > (double)s - 1e-16 (TD/Trixel.cu:157).
RT_HD bool gt_eps_ref(float a, float s) { return (double)a > (double)s - kEps; }
RT_HD bool gt_eps(float a, float s) {
#ifndef RT_FAST_PREDICATES
    return gt_eps_ref(a, s);
#endif
    if (a != s && fabsf(s) >= kSmall) return a > s;
    return gt_eps_ref(a, s);
}

// (float)((double)s + 1e-16) (TD/Trixel.cu:150 with a zero object offset).
RT_HD float add_eps_ref(float s) { return (float)((double)s + kEps); }
RT_HD float add_eps(float s) {
#ifndef RT_FAST_PREDICATES
    return add_eps_ref(s);
#endif
    return fabsf(s) >= kSmall ? s : add_eps_ref(s);
}

// Guarded float forms: the double tests above reduced to one float compare,
// exact whenever the guard holds (tests/predicates_check.cpp checks them on
// edge sets and random sweeps).  The traversal evaluates the guards of a
// whole node visit at once and takes these forms when every guard holds,
// which is every visit of a camera more than ~1e-6 away from split planes
// and box faces; otherwise it takes the double forms.
//   split_safe(s): |s| >= 2^-20 or NaN  -> add_eps(s) == s and, for a != s,
//                  lt_eps(a, s) == (a < s), gt_eps(a, s) == (a > s)
//                  (at a == s the answer depends on whether 1e-16 exceeds
//                  half a double ulp of s: the double form decides)
//   entry_safe(m): m <= -eps_f() or m >= 2^-20 or NaN -> enter(m, t) == (m > -eps_f() && t >= m)
//                  (t >= fl64(m - 1e-16) with fl64(m - 1e-16) in (pred(m), m])
RT_HD bool split_safe(float s) { return !(fabsf(s) < kSmall); }
RT_HD bool entry_safe(float m) { return !(m > -eps_f() && m < kSmall); }
RT_HD bool lt_eps_f(float a, float s) { return a < s; }
RT_HD bool gt_eps_f(float a, float s) { return a > s; }
RT_HD bool enter_f(float maxt0, float mint1) { return maxt0 > -eps_f() && mint1 >= maxt0; }

// Exact float forms of lt_eps_ref / gt_eps_ref with the equality case
// decided too (round 6: the translated and shadow kFast walks, whose split
// values s = s2 + ds are computed per visit, so no threshold can be stored in
// the record).  For |s| >= 2^-20 no float lies strictly between s and
// s +/- 1e-16, so for a != s the test is a < s (a > s); at a == s it is
// whether the double sum s + 1e-16 rounds above s (s - 1e-16 below s): the
// double spacing beyond s must be below 2e-16, which holds exactly when
// |s| < 1, or s == -1 (s == +1) whose spacing toward zero is half the
// spacing of its binade.  Valid for every float a and every s with
// |s| >= 2^-20, infinities and NaN included (tests/predicates_check.cpp).
RT_HD bool lt_eps_x(float a, float s) { return a < s || (a == s && (fabsf(s) < 1.0f || s == -1.0f)); }
RT_HD bool gt_eps_x(float a, float s) { return a > s || (a == s && (fabsf(s) < 1.0f || s == 1.0f)); }

}  // namespace pred
}  // namespace rt
