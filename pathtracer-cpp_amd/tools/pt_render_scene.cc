// pt_render_scene — renders a .ptscene through the C++ drop-in API
// (pathtracer/pathtracer.h) and writes the linear float32 image (h = 0 first).
// Used by the GPU tests to check that the C++ host path (Camera, BVH::build,
// pt_render_into -> libpt_hip.so) is bit-identical to the reference.
//
//   pt_render_scene <scene.ptscene> <spp> <depth> <out.f32> [W H]
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>

#include "pathtracer/pathtracer.h"

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s scene.ptscene spp depth out.f32 [W H]\n", argv[0]);
        return 2;
    }
    std::ifstream in(argv[1]);
    if (!in) {
        std::fprintf(stderr, "cannot open %s\n", argv[1]);
        return 2;
    }
    BVH bvh;
    vec3 pos(0), fwd(0), up(0);
    int rx = 0, ry = 0;
    double fov_deg = 0, dist = 1;
    std::string line;
    auto F = [](std::istringstream& s) { double d; s >> d; return (float)d; };
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string tag;
        if (!(ls >> tag) || tag[0] == '#') continue;
        if (tag == "camera") {
            float v[9];
            for (float& x : v) x = F(ls);
            ls >> rx >> ry >> fov_deg >> dist;
            pos = vec3(v[0], v[1], v[2]);
            fwd = vec3(v[3], v[4], v[5]);
            up = vec3(v[6], v[7], v[8]);
        } else if (tag == "tri") {
            float v[9], c[7];
            int type;
            for (float& x : v) x = F(ls);
            ls >> type;
            for (float& x : c) x = F(ls);
            bvh.add_triangle(Triangle(vec3(v[0], v[1], v[2]), vec3(v[3], v[4], v[5]), vec3(v[6], v[7], v[8]),
                                      Material((Material::Type)type, vec3(c[0], c[1], c[2]),
                                               vec3(c[3], c[4], c[5]), c[6])));
        }
    }
    if (argc >= 7) {
        rx = std::atoi(argv[5]);
        ry = std::atoi(argv[6]);
    }
    Camera camera(pos, fwd, up, ivec2(rx, ry), fov_deg * M_PI / 180, (float)dist);
    bvh.build();
    Image image;
    pt_stats st;
    pt_render_into(camera, bvh, std::atoi(argv[2]), std::atoi(argv[3]), image, &st);
    FILE* fp = std::fopen(argv[4], "wb");
    if (!fp) return 2;
    for (int h = 0; h < ry; h++)
        for (int w = 0; w < rx; w++) std::fwrite(&image.pixels[h][w], sizeof(float), 3, fp);
    std::fclose(fp);
    std::printf("{\"rays\": %llu, \"kernel_ms\": %.3f}\n", (unsigned long long)st.rays, st.kernel_ms);
    return 0;
}
