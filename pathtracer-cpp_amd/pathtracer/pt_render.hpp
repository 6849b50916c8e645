// pt_render.hpp — render entry points of the drop-in API (reference: pathtracer/render.h).
//
// render_cpu (render.h:62-104) and render_gpu (render.h:109-152) keep their
// signatures, console lines, messages and bool results; both hand the built BVH to
// libpt_hip.so, which runs the per-pixel trace loop on every visible GPU, gathers the
// row bands on the first one and applies gamma_correct(2.2) + save_png's quantisation
// there (pt_render_rgb8_devices): the host receives the PNG's bytes (3 B per pixel
// instead of 12) and writes them. The per-row (render.h:87) / per-chunk (render.h:136)
// progress lines follow the library's progress reports. The OpenGL tile path and the
// SFML viewer (render_realtime) are not part of this framework.
#pragma once

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "pt_camera.hpp"
#include "pt_hip.h"
#include "pt_image.hpp"
#include "pt_scene.hpp"

#ifndef SHIFT_BIAS
#define SHIFT_BIAS 1e-4
#endif

struct Timer {
    std::chrono::time_point<std::chrono::high_resolution_clock> start_time;
    void start() { start_time = std::chrono::high_resolution_clock::now(); }
    void reset() { start(); }
    float seconds() {
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
            std::chrono::high_resolution_clock::now() - start_time);
        return ms.count() / 1000.0f;
    }
};

inline int ceildiv(int a, int b) { return (a + b - 1) / b; }

// The devices a render runs on: every visible GPU, or PT_DEVICES="0,2,...".
inline std::vector<int32_t> pt_render_devices() {
    std::vector<int32_t> devs;
    if (const char* e = std::getenv("PT_DEVICES")) {
        std::stringstream ss(e);
        for (std::string tok; std::getline(ss, tok, ',');)
            if (!tok.empty()) devs.push_back((int32_t)std::atoi(tok.c_str()));
    }
    for (int d = 0, n = pt_device_count(); devs.empty() && d < n; d++) devs.push_back(d);
    if (devs.empty()) devs.push_back(0);
    return devs;
}

// The scene and parameters of one render (views of `bvh`'s arrays, kept alive here).
struct PtRenderCall {
    std::vector<float> verts;
    std::vector<pt_material> mats;
    pt_scene sc;
    pt_camera cam;
    pt_params prm;
    PtRenderCall(const Camera& camera, BVH& bvh, int samples, int depth, unsigned seed)
        : verts(bvh.packed_vertices()), mats(bvh.packed_materials()) {
        sc.num_tris = (int32_t)bvh.triangles.size();
        sc.verts = verts.data();
        sc.materials = mats.data();
        sc.num_nodes = (int32_t)bvh.nodes.size();
        sc.nodes = reinterpret_cast<const pt_bvh_node*>(bvh.nodes.data());
        sc.tri_idx = bvh.tri_idx.data();
        cam = camera.to_c();
        std::memset(&prm, 0, sizeof(prm));
        prm.spp = samples;
        prm.depth = depth;
        prm.seed = seed;
        prm.part_count = 1;
        prm.band_rows = 1;  // rows dealt across the devices one at a time (best balance: DESIGN.md §6)
    }
};

// Render `bvh` through libpt_hip.so into `image` (linear mean, pixels[h][w]).
// Throws std::runtime_error on a device error, as the reference's GL path does.
inline bool pt_render_into(const Camera& camera, BVH& bvh, int samples, int depth, Image& image,
                           pt_stats* stats = nullptr, unsigned seed = SEED) {
    PtRenderCall call(camera, bvh, samples, depth, seed);
    std::vector<float> out((size_t)camera.res.x * camera.res.y * 3);
    pt_stats st;
    const std::vector<int32_t> devs = pt_render_devices();
    const int rc = pt_render_f32_devices(&call.sc, &call.cam, &call.prm, devs.data(), (int32_t)devs.size(),
                                         out.data(), &st);
    if (rc != PT_OK) throw std::runtime_error(std::string("libpt_hip: ") + pt_last_error());
    image = Image(camera.res);
    for (int h = 0; h < camera.res.y; h++)
        for (int w = 0; w < camera.res.x; w++) {
            const float* p = &out[((size_t)h * camera.res.x + w) * 3];
            image.pixels[h][w] = vec3(p[0], p[1], p[2]);
        }
    if (stats) *stats = st;
    return true;
}

// The reference's progress lines, "\rRendered: k/N rows." (render.h:87) or "... chunks."
// (render.h:136) for k = 1..N in order, advanced as the library reports progress.
struct PtProgressLines {
    const char* unit;
    int total;
    int printed = 0;
    void advance(int k) {
        while (printed < k && printed < total) {
            ++printed;
            std::cout << "\rRendered: " << printed << '/' << total << ' ' << unit << '.' << std::flush;
        }
    }
};

inline void pt_progress_lines(void* user, int64_t done, int64_t total) {
    PtProgressLines* p = static_cast<PtProgressLines*>(user);
    p->advance(total > 0 ? (int)((long double)done * p->total / total) : p->total);
}

// Render through libpt_hip.so; gamma_correct(2.2) and save_png's quantisation run on the
// device: returns the PNG's RGB bytes, top row first (image.h:45-56).
inline std::vector<unsigned char> pt_render_png_bytes(const Camera& camera, BVH& bvh, int samples, int depth,
                                                      PtProgressLines* lines, pt_stats* stats = nullptr,
                                                      unsigned seed = SEED) {
    PtRenderCall call(camera, bvh, samples, depth, seed);
    if (lines) {
        call.prm.progress = pt_progress_lines;
        call.prm.progress_user = lines;
    }
    std::vector<unsigned char> rgb((size_t)camera.res.x * camera.res.y * 3);
    pt_stats st;
    const std::vector<int32_t> devs = pt_render_devices();
    const int rc = pt_render_rgb8_devices(&call.sc, &call.cam, &call.prm, devs.data(), (int32_t)devs.size(),
                                          (float)2.2, rgb.data(), &st);
    if (rc != PT_OK) throw std::runtime_error(std::string("libpt_hip: ") + pt_last_error());
    if (stats) *stats = st;
    return rgb;
}

// Image::save_png's file write (image.h:59-61) for bytes already quantised.
inline void pt_save_png_bytes(const std::string& filename, const std::vector<unsigned char>& rgb, const ivec2& res) {
    if (pt_write_png(filename.c_str(), rgb.data(), res.x, res.y) != PT_OK)
        std::cerr << "Failed to write image to file: " << filename << '\n';
}

inline bool pt_prepare(BVH& bvh) {
    if (bvh.empty()) {
        std::cerr << "No triangles in scene.\n";
        return false;
    }
    if (!bvh.built) {
        std::cerr << "Bounding volume heirarchy not built.\nBuilding...\n";
        bvh.build();
    }
    return true;
}

inline void pt_print_done(float seconds, const char* tail) {
    std::ios old_state(nullptr);
    old_state.copyfmt(std::cout);
    std::cout << std::fixed << std::setprecision(2);
    std::cout << "\nDone in " << seconds << " seconds." << tail;
    std::cout.copyfmt(old_state);
}

inline bool render_cpu(const Camera& camera, BVH& bvh, int samples, int depth, const std::string& filename) {
    if (!pt_prepare(bvh)) return false;
    Timer timer;
    timer.start();
    std::cout << "Rendered: 0/" << camera.res.y << " rows.";
    PtProgressLines lines{"rows", camera.res.y};
    const std::vector<unsigned char> rgb = pt_render_png_bytes(camera, bvh, samples, depth, &lines);
    lines.advance(camera.res.y);
    pt_print_done(timer.seconds(), "\nColor correcting...\n");
    pt_save_png_bytes(filename, rgb, camera.res);
    std::cout << "Saved to " << filename << '\n';
    return true;
}

inline bool render_gpu(const Camera& camera, BVH& bvh, int samples, int depth, const ivec2& chunk_size,
                       const std::string& filename) {
    if (!pt_prepare(bvh)) return false;
    // the device work is not tiled (a persistent kernel needs no watchdog-sized draws);
    // chunk_size sets the progress lines' count, as the reference's tile loop would
    const int total = ceildiv(camera.res.x, chunk_size.x) * ceildiv(camera.res.y, chunk_size.y);
    Timer timer;
    timer.start();
    std::cout << "Rendered: 0/" << total << " chunks.";
    PtProgressLines lines{"chunks", total};
    const std::vector<unsigned char> rgb = pt_render_png_bytes(camera, bvh, samples, depth, &lines);
    lines.advance(total);
    pt_print_done(timer.seconds(), "\n");
    pt_save_png_bytes(filename, rgb, camera.res);
    std::cout << "Saved to " << filename << '\n';
    return true;
}
