// pt_render.hpp — render entry points of the drop-in API (reference: pathtracer/render.h).
//
// render_cpu (render.h:62-104) and render_gpu (render.h:109-152) keep their
// signatures, messages and bool results; both hand the built BVH to
// libpt_hip.so (pt_render_f32), which runs the per-pixel trace loop on the GPU
// and returns the linear mean image after /spp. Gamma 2.2 and the PNG write
// follow on the host exactly as in the reference. The OpenGL tile path and the
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

// Render `bvh` through libpt_hip.so into `image` (linear mean, pixels[h][w]).
// Throws std::runtime_error on a device error, as the reference's GL path does.
inline bool pt_render_into(const Camera& camera, BVH& bvh, int samples, int depth, Image& image,
                           pt_stats* stats = nullptr, unsigned seed = SEED) {
    const std::vector<float> verts = bvh.packed_vertices();
    const std::vector<pt_material> mats = bvh.packed_materials();
    pt_scene sc;
    sc.num_tris = (int32_t)bvh.triangles.size();
    sc.verts = verts.data();
    sc.materials = mats.data();
    sc.num_nodes = (int32_t)bvh.nodes.size();
    sc.nodes = reinterpret_cast<const pt_bvh_node*>(bvh.nodes.data());
    sc.tri_idx = bvh.tri_idx.data();
    const pt_camera cam = camera.to_c();
    pt_params prm;
    std::memset(&prm, 0, sizeof(prm));
    prm.spp = samples;
    prm.depth = depth;
    prm.seed = seed;
    prm.part_count = 1;
    prm.band_rows = 1;
    std::vector<float> out((size_t)camera.res.x * camera.res.y * 3);
    pt_stats st;
    // Every visible GPU (PT_DEVICES="0,2,..." picks them), row bands dealt across them.
    std::vector<int32_t> devs;
    if (const char* e = std::getenv("PT_DEVICES")) {
        std::stringstream ss(e);
        for (std::string tok; std::getline(ss, tok, ',');)
            if (!tok.empty()) devs.push_back((int32_t)std::atoi(tok.c_str()));
    }
    for (int d = 0, n = pt_device_count(); devs.empty() && d < n; d++) devs.push_back(d);
    if (devs.empty()) devs.push_back(0);
    prm.band_rows = 8;
    const int rc = pt_render_f32_devices(&sc, &cam, &prm, devs.data(), (int32_t)devs.size(), out.data(), &st);
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
    Image image;
    Timer timer;
    timer.start();
    std::cout << "Rendered: 0/" << camera.res.y << " rows.";
    pt_render_into(camera, bvh, samples, depth, image);
    std::cout << "\rRendered: " << camera.res.y << '/' << camera.res.y << " rows." << std::flush;
    pt_print_done(timer.seconds(), "\nColor correcting...\n");
    image.gamma_correct(2.2);
    image.save_png(filename);
    std::cout << "Saved to " << filename << '\n';
    return true;
}

inline bool render_gpu(const Camera& camera, BVH& bvh, int samples, int depth, const ivec2& chunk_size,
                       const std::string& filename) {
    if (!pt_prepare(bvh)) return false;
    const int total = ceildiv(camera.res.x, chunk_size.x) * ceildiv(camera.res.y, chunk_size.y);
    Image image;
    Timer timer;
    timer.start();
    std::cout << "Rendered: 0/" << total << " chunks.";
    pt_render_into(camera, bvh, samples, depth, image);
    std::cout << "\rRendered: " << total << '/' << total << " chunks." << std::flush;
    pt_print_done(timer.seconds(), "\n");
    image.gamma_correct(2.2);
    image.save_png(filename);
    std::cout << "Saved to " << filename << '\n';
    return true;
}
