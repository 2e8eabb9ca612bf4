// CPU check of rt_predicates.h: every fast single-precision form against the
// reference's double form (built and run by tests/test_predicates.py).
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "../cpp_cuda_raytracer_dev_amd/csrc/rt_predicates.h"

using namespace rt::pred;

static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
    const long n_random = argc > 1 ? atol(argv[1]) : 20000000;
    std::vector<float> edge;
    const float specials[] = {0.0f, -0.0f, 1.0f, -1.0f, 2.0f, -2.0f, 0.5f, -0.5f, kSmall, -kSmall, 1e-16f, -1e-16f,
                              eps_f(), -eps_f(), 1e-30f, -1e-30f, bits(1), bits(0x80000001u), bits(0x00800000u),
                              __builtin_inff(), -__builtin_inff(), __builtin_nanf(""), 400.0f, -400.0f, 3.0e38f};
    for (float s : specials) edge.push_back(s);
    for (int e = -149; e <= 127; e++) {  // powers of two and their neighbours, both signs
        const float p = ldexpf(1.0f, e);
        for (float v : {p, -p}) {
            const uint32_t u = ubits(v);
            for (int d = -2; d <= 2; d++) edge.push_back(bits(u + d));
        }
    }
    long bad = 0, checked = 0, guarded = 0;
    auto check = [&](float a, float b) {
        checked++;
        if (enter(a, b) != enter_ref(a, b)) { if (bad++ < 10) printf("enter %a %a\n", a, b); }
        if (lt_eps(a, b) != lt_eps_ref(a, b)) { if (bad++ < 10) printf("lt_eps %a %a\n", a, b); }
        if (gt_eps(a, b) != gt_eps_ref(a, b)) { if (bad++ < 10) printf("gt_eps %a %a\n", a, b); }
        const float x = add_eps(a), y = add_eps_ref(a);
        if (ubits(x) != ubits(y) && !(x != x && y != y)) { if (bad++ < 10) printf("add_eps %a\n", a); }
        // the guarded float forms of the traversal (rt_predicates.h)
        if (split_safe(b) && a != b) {
            if (lt_eps_f(a, b) != lt_eps_ref(a, b)) { if (bad++ < 10) printf("lt_eps_f %a %a\n", a, b); }
            if (gt_eps_f(a, b) != gt_eps_ref(a, b)) { if (bad++ < 10) printf("gt_eps_f %a %a\n", a, b); }
            guarded++;
        }
        if (split_safe(a) && ubits(a) != ubits(add_eps_ref(a)) && !(a != a)) {
            if (bad++ < 10) printf("add_eps_f %a\n", a);
        }
        if (entry_safe(a) && enter_f(a, b) != enter_ref(a, b)) { if (bad++ < 10) printf("enter_f %a %a\n", a, b); }
        // the per-visit forms of the translated / shadow kFast walks (equal operands included)
        if (!(fabsf(b) < kSmall)) {
            if (lt_eps_x(a, b) != lt_eps_ref(a, b)) { if (bad++ < 10) printf("lt_eps_x %a %a\n", a, b); }
            if (gt_eps_x(a, b) != gt_eps_ref(a, b)) { if (bad++ < 10) printf("gt_eps_x %a %a\n", a, b); }
            if (lt_eps_x(b, b) != lt_eps_ref(b, b)) { if (bad++ < 10) printf("lt_eps_x= %a\n", b); }
            if (gt_eps_x(b, b) != gt_eps_ref(b, b)) { if (bad++ < 10) printf("gt_eps_x= %a\n", b); }
        }
    };
    for (float a : edge)
        for (float b : edge) check(a, b);
    std::mt19937_64 rng(20221015);
    for (long i = 0; i < n_random; i++) {
        const uint64_t r = rng();
        const float a = bits((uint32_t)r);
        float b;
        switch ((r >> 32) & 3) {
        case 0: b = bits((uint32_t)(r >> 32)); break;              // independent
        case 1: b = bits(ubits(a) + (int32_t)((r >> 34) % 5) - 2); break;  // neighbours
        case 2: b = a; break;                                      // equal
        default: b = -a; break;
        }
        check(a, b);
        check(b, a);
    }
    printf("checked %ld pairs (%ld under split guards), %ld mismatches\n", checked, guarded, bad);
    return bad != 0;
}
