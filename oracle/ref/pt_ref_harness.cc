// pt_ref_harness.cc — TEST INFRASTRUCTURE ONLY (oracle/_ref). Never shipped,
// never linked into libpt_hip.so.
//
// Drives the UNMODIFIED reference CPU path (Blackgaurd/pathtracer-cpp):
//   trace()         render.h:36-61      (extracted verbatim at build time,
//   render_cpu()    render.h:62-104      render.h:16-108, see build_ref.sh)
//   BVH::build      bvh.h:79-155, BVH::intersect bvh.h:156-183, load_obj 184-242
//   Camera          camera.h:33-73, Image image.h, lcg rng.h
// compiled by g++ -O3 from the files under /root/reference. The only thing
// this file adds is the driver loop: the scene comes from a .ptscene text file
// (tests/golden/scenes.py writes it), and — unless --global-rng is given — the
// global LCG is re-seeded before each sample with pt_sample_seed() (the
// stream policy of include/pt_hip.h). The loop body is render.h:83-84.
//
// Outputs raw little-endian float32 buffers (linear, after /spp).
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iomanip>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>
#include <cmath>

#include "pathtracer/bvh.h"
#include "pathtracer/camera.h"
#include "pathtracer/image.h"
#include "render_cpu_part.h"  // render.h:16-108, extracted by build_ref.sh

#include "pt_hip.h"  // pt_sample_seed (stream policy) only

namespace {

struct Args {
    std::string scene, out, pixels, dump_bvh, load_bvh, dump_tris, png, obj, mtl = "./";
    int res_x = -1, res_y = -1, spp = 16, depth = 5;
    unsigned seed = PT_SEED;
    bool global_rng = false, quiet = false;
    int row_begin = 0, row_end = -1;  // rows [row_begin, row_end) for bounded timing samples
};

[[noreturn]] void die(const std::string& m) {
    std::fprintf(stderr, "pt_ref: %s\n", m.c_str());
    std::exit(2);
}

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; i++) {
        std::string k = argv[i];
        auto need = [&]() -> std::string {
            if (i + 1 >= argc) die("missing value for " + k);
            return argv[++i];
        };
        if (k == "--scene") a.scene = need();
        else if (k == "--obj") a.obj = need();
        else if (k == "--mtl") a.mtl = need();
        else if (k == "--out") a.out = need();
        else if (k == "--pixels") a.pixels = need();
        else if (k == "--dump-bvh") a.dump_bvh = need();
        else if (k == "--load-bvh") a.load_bvh = need();
        else if (k == "--dump-tris") a.dump_tris = need();
        else if (k == "--png") a.png = need();
        else if (k == "--res") { a.res_x = std::atoi(need().c_str()); a.res_y = std::atoi(need().c_str()); }
        else if (k == "--spp") a.spp = std::atoi(need().c_str());
        else if (k == "--depth") a.depth = std::atoi(need().c_str());
        else if (k == "--seed") a.seed = (unsigned)std::strtoul(need().c_str(), nullptr, 0);
        else if (k == "--rows") { a.row_begin = std::atoi(need().c_str()); a.row_end = std::atoi(need().c_str()); }
        else if (k == "--global-rng") a.global_rng = true;
        else if (k == "--quiet") a.quiet = true;
        else die("unknown option " + k);
    }
    if (a.scene.empty()) die("--scene is required");
    return a;
}

// .ptscene: "camera px py pz fx fy fz ux uy uz res_x res_y fov_deg distance"
//           "tri x1 y1 z1 x2 y2 z2 x3 y3 z3 type cr cg cb er eg eb rough"
// Numbers are parsed as double then narrowed to float — the same two roundings a
// double literal passed to vec3(float...) undergoes in the reference examples.
struct CamSpec { vec3 pos, fwd, up; int rx, ry; double fov_deg; float dist; };

float F(std::istringstream& in) { double d; in >> d; return (float)d; }

CamSpec load_scene(const std::string& path, BVH& bvh) {
    std::ifstream f(path);
    if (!f) die("cannot open " + path);
    CamSpec cs{};
    bool have_cam = false;
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream in(line);
        std::string tag;
        if (!(in >> tag) || tag[0] == '#') continue;
        if (tag == "camera") {
            float v[9];
            for (float& x : v) x = F(in);
            in >> cs.rx >> cs.ry >> cs.fov_deg;
            cs.dist = F(in);
            cs.pos = vec3(v[0], v[1], v[2]);
            cs.fwd = vec3(v[3], v[4], v[5]);
            cs.up = vec3(v[6], v[7], v[8]);
            have_cam = true;
        } else if (tag == "tri") {
            float v[9];
            for (float& x : v) x = F(in);
            int type;
            in >> type;
            float c[7];
            for (float& x : c) x = F(in);
            Material m((Material::Type)type, vec3(c[0], c[1], c[2]), vec3(c[3], c[4], c[5]), c[6]);
            bvh.add_triangle(Triangle(vec3(v[0], v[1], v[2]), vec3(v[3], v[4], v[5]),
                                      vec3(v[6], v[7], v[8]), m));
        } else {
            die("bad scene line: " + line);
        }
    }
    if (!have_cam) die("scene has no camera line");
    return cs;
}

void write_f32(const std::string& path, const std::vector<float>& v) {
    FILE* fp = std::fopen(path.c_str(), "wb");
    if (!fp) die("cannot write " + path);
    std::fwrite(v.data(), sizeof(float), v.size(), fp);
    std::fclose(fp);
}

}  // namespace

int main(int argc, char** argv) {
    Args a = parse(argc, argv);
    BVH bvh;
    CamSpec cs = load_scene(a.scene, bvh);
    if (!a.obj.empty()) bvh.load_obj(a.obj, a.mtl);
    if (!a.dump_tris.empty()) {  // int32 n, then per triangle v1, v2, v3 (9 floats) + Material (32 B)
        FILE* fp = std::fopen(a.dump_tris.c_str(), "wb");
        if (!fp) die("cannot write " + a.dump_tris);
        static_assert(sizeof(Material) == 32, "reference Material layout");
        int32_t n = (int32_t)bvh.triangles.size();
        std::fwrite(&n, 4, 1, fp);
        for (const Triangle& t : bvh.triangles) {
            const float v[9] = {t.v1.x, t.v1.y, t.v1.z, t.v2.x, t.v2.y, t.v2.z, t.v3.x, t.v3.y, t.v3.z};
            std::fwrite(v, 4, 9, fp);
            std::fwrite(&t.material, sizeof(Material), 1, fp);
        }
        std::fclose(fp);
    }
    if (a.res_x > 0) { cs.rx = a.res_x; cs.ry = a.res_y; }
    // fov argument exactly as `60 * DEG2RAD` in the examples: (deg * M_PI) / 180, narrowed.
    Camera camera(cs.pos, cs.fwd, cs.up, ivec2(cs.rx, cs.ry), cs.fov_deg * M_PI / 180, cs.dist);

    auto tb = std::chrono::steady_clock::now();
    if (!a.load_bvh.empty()) {
        // A tree in the --dump-bvh format (e.g. the fast builder's, proven bit-identical to
        // BVH::build by its sha256): fills the reference BVH's own public arrays, so the
        // O(n^2) build (380 s for the 99k-triangle mesh) is skipped; trace() is unchanged.
        FILE* fp = std::fopen(a.load_bvh.c_str(), "rb");
        if (!fp) die("cannot open " + a.load_bvh);
        int32_t n = 0, t = 0;
        if (std::fread(&n, 4, 1, fp) != 1 || std::fread(&t, 4, 1, fp) != 1 || n <= 0 ||
            t != (int32_t)bvh.triangles.size())
            die("bad --load-bvh header");
        bvh.nodes.resize(n);
        bvh.tri_idx.resize(t);
        if (std::fread(bvh.nodes.data(), sizeof(BVHNode), n, fp) != (size_t)n ||
            std::fread(bvh.tri_idx.data(), 4, t, fp) != (size_t)t)
            die("short --load-bvh file");
        std::fclose(fp);
        bvh.built = true;
    } else {
        bvh.build();
    }
    double build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count();

    if (!a.dump_bvh.empty()) {
        FILE* fp = std::fopen(a.dump_bvh.c_str(), "wb");
        if (!fp) die("cannot write " + a.dump_bvh);
        static_assert(sizeof(BVHNode) == 40, "reference BVHNode layout");
        int32_t n = (int32_t)bvh.nodes.size(), t = (int32_t)bvh.tri_idx.size();
        std::fwrite(&n, 4, 1, fp);
        std::fwrite(&t, 4, 1, fp);
        std::fwrite(bvh.nodes.data(), sizeof(BVHNode), n, fp);
        std::fwrite(bvh.tri_idx.data(), 4, t, fp);
        std::fclose(fp);
    }

    const int W = cs.rx, H = cs.ry;
    vec3 ray_o, ray_d;
    if (!a.pixels.empty()) {
        // Sampled pixels at full spp: one "w h" per line.
        std::ifstream pf(a.pixels);
        std::vector<float> out;
        int w, h;
        auto t0 = std::chrono::steady_clock::now();
        while (pf >> w >> h) {
            vec3 acc(0, 0, 0);
            for (int s = 0; s < a.spp; s++) {
                rng.seed(pt_sample_seed((uint32_t)(h * W + w), (uint32_t)s, a.seed));
                camera.get_ray(w, h, ray_o, ray_d);
                acc += trace(bvh, ray_o, ray_d, a.depth);
            }
            acc /= (float)a.spp;
            out.push_back(acc.x);
            out.push_back(acc.y);
            out.push_back(acc.z);
        }
        double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!a.out.empty()) write_f32(a.out, out);
        std::printf("{\"pixels\": %zu, \"render_s\": %.6f, \"build_s\": %.6f}\n", out.size() / 3, sec,
                    build_s);
        return 0;
    }

    if (a.row_end < 0) a.row_end = H;
    Image image(camera.res);
    auto t0 = std::chrono::steady_clock::now();
    // render.h:80-88 with the per-sample reseed (or the untouched global stream).
    for (int h = a.row_begin; h < a.row_end; h++) {
        for (int w = 0; w < W; w++) {
            for (int s = 0; s < a.spp; s++) {
                if (!a.global_rng) rng.seed(pt_sample_seed((uint32_t)(h * W + w), (uint32_t)s, a.seed));
                camera.get_ray(w, h, ray_o, ray_d);
                image.get_pixel(w, h) += trace(bvh, ray_o, ray_d, a.depth);
            }
        }
    }
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    image /= a.spp;  // render.h:97

    if (!a.out.empty()) {
        std::vector<float> out;
        out.reserve((size_t)(a.row_end - a.row_begin) * W * 3);
        for (int h = a.row_begin; h < a.row_end; h++)
            for (int w = 0; w < W; w++) {
                const vec3& p = image.pixels[h][w];
                out.push_back(p.x);
                out.push_back(p.y);
                out.push_back(p.z);
            }
        write_f32(a.out, out);
    }
    if (!a.png.empty()) {
        image.gamma_correct(2.2);  // render.h:99
        image.save_png(a.png);     // render.h:100
    }
    std::printf(
        "{\"res\": [%d, %d], \"rows\": [%d, %d], \"spp\": %d, \"depth\": %d, \"render_s\": %.6f, "
        "\"build_s\": %.6f, \"nodes\": %zu, \"tris\": %zu}\n",
        W, H, a.row_begin, a.row_end, a.spp, a.depth, sec, build_s, bvh.nodes.size(), bvh.size());
    return 0;
}
