// rt_headless.cpp -- the headless frame loop that replaces WinMain
// (TD/WinMain.cpp:44-249), written against the reference-shaped C++ facade.
//
//   rt_headless <mesh.ply> <mode 0|1|2> [w h frames out.ppm flat keys]
//
// keys: held keys per frame, cycled, one input tick per frame (WinMain ticks
// at TICK_RATE, :173): letters of R W S Q E T, '+' joins keys held together,
// '.' is a tick with none, e.g. "WWR+W.Q".
// Same construction sequence as WinMain: Camera (:69-74), read_ply (:93),
// Color (:114-121), Trixel + set_sorted_voxels + create_kd (:134-144), two
// Objects added to the camera (:152-156), then render + color_pixels per
// frame (:212-213).  Prints load / build / frame timings and writes the last
// frame as a binary PPM (top row first).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_facade.hpp"

using namespace rtmi;

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s mesh.ply mode [w h frames out.ppm flat]\n", argv[0]);
        return 2;
    }
    const char* mesh = argv[1];
    const u8 mode = (u8)std::atoi(argv[2]);
    const s32 w = argc > 3 ? std::atoi(argv[3]) : 960, h = argc > 4 ? std::atoi(argv[4]) : 540;
    const int frames = argc > 5 ? std::atoi(argv[5]) : 100;
    const char* out = argc > 6 ? argv[6] : nullptr;
    const u32 render_mode = (argc > 7 && std::atoi(argv[7])) ? RENDER_MODE_FLAT : RENDER_MODE_KD;
    std::vector<uint32_t> ticks;  // held-key masks, one per frame
    if (argc > 8) {
        uint32_t m = 0;
        for (const char* k = argv[8];; k++) {
            const char c = *k;
            if (c == '+') continue;
            m |= c == 'R' ? RT_KEY_R : c == 'W' ? RT_KEY_W : c == 'S' ? RT_KEY_S : c == 'Q' ? RT_KEY_Q
               : c == 'E' ? RT_KEY_E : c == 'T' ? RT_KEY_T : 0u;
            if (c == '\0' || k[1] != '+') {
                if (c != '\0' || m) ticks.push_back(m);
                m = 0;
            }
            if (c == '\0') break;
        }
    }

    Camera* main_cam = new Camera(w, h, film_w(w, h), (T_fp).024, (T_fp).055, (T_fp)0.0, (T_fp)0.10, (T_fp)-1.0,
                                  (T_fp)0.00, (T_fp)0.100, (T_fp)0.00, (T_fp)0.0, (T_fp)1.0, (T_fp)0.0);
    if (main_cam->status) { std::fprintf(stderr, "Camera: %s\n", rt_last_error_string()); return 1; }

    T_fp* points = nullptr;
    kd_leaf_sort* leafs = nullptr;
    kd_vertex* verts = nullptr;
    T_uint ntri = 0, nvert = 0;
    double t0 = now_s();
    if (read_ply(mesh, &points, &ntri, &leafs, &verts, &nvert, mode)) {
        std::fprintf(stderr, "read_ply: %s\n", rt_last_error_string());
        return 1;
    }
    std::printf("Time to Read Tree: %f seconds\n\t\t primitives: %u\n", now_s() - t0, ntri);

    Color color;
    std::vector<Color::radiance> rad(ntri, Color::radiance{(T_fp).1, (T_fp).55, (T_fp).20});
    color.rad = rad.data();

    double t1 = now_s();
    Trixel* trixel_list = new Trixel(ntri, points, &color);
    if (trixel_list->status) { std::fprintf(stderr, "Trixel: %s\n", rt_last_error_string()); return 1; }
    trixel_list->set_sorted_voxels(leafs, ntri);
    if (trixel_list->create_kd()) { std::fprintf(stderr, "create_kd: %s\n", rt_last_error_string()); return 1; }
    std::printf("Total Time to build tree: %f seconds\n", now_s() - t1);
    rt_host_free(points);
    rt_host_free(leafs);

    Object* obj1 = new Object(trixel_list);
    Object* obj2 = new Object(trixel_list);
    if (main_cam->add_object(obj1) || main_cam->add_object(obj2)) {
        std::fprintf(stderr, "add_object: %s\n", rt_last_error_string());
        return 1;
    }

    // warm up, then time `frames` frames of render + D2H (the reference's FPS loop)
    obj1->render(main_cam, render_mode);
    main_cam->color_pixels(PHONG_COLOR_TAG);
    double t2 = now_s();
    for (int f = 0; f < frames; f++) {
        if (!ticks.empty() && obj1->key_tick(ticks[(size_t)f % ticks.size()])) {
            std::fprintf(stderr, "transform: %s\n", rt_last_error_string());
            return 1;
        }
        if (obj1->render(main_cam, render_mode)) { std::fprintf(stderr, "render: %s\n", rt_last_error_string()); return 1; }
        if (main_cam->color_pixels(PHONG_COLOR_TAG)) {
            std::fprintf(stderr, "color_pixels: %s\n", rt_last_error_string());
            return 1;
        }
    }
    const double dt = (now_s() - t2) / frames;
    std::printf("Resolution: %d x %d\nFPS (%srender + D2H): %f\n", w, h, ticks.empty() ? "" : "key tick + ",
                1.0 / dt);

    if (out) {
        FILE* fp = std::fopen(out, "wb");
        if (!fp) { std::perror(out); return 1; }
        std::fprintf(fp, "P6\n%d %d\n255\n", w, h);
        for (s32 y = h - 1; y >= 0; y--)  // the DIB is bottom-up (TD/WinMain.cpp:32)
            for (s32 x = 0; x < w; x++) {
                const u32 c = main_cam->h_mem.h_color.c[(size_t)y * w + x];
                const unsigned char px[3] = {(unsigned char)(c >> 16), (unsigned char)(c >> 8), (unsigned char)c};
                std::fwrite(px, 1, 3, fp);
            }
        std::fclose(fp);
    }
    delete obj1;
    delete obj2;
    delete main_cam;
    delete trixel_list;
    return 0;
}
