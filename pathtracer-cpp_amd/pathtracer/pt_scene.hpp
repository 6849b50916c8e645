// pt_scene.hpp — scene types of the drop-in API.
// Reference: rng.h (lcg, global rng), aabb.h (AABB), material.h (Material, BRDF
// samplers), triangle.h (Triangle), bvh.h (BVHNode, BVH). Memory layouts of
// BVHNode (40 B) and Material (32 B) equal the reference's and the C ABI's
// pt_bvh_node / pt_material, so a built BVH is handed to libpt_hip.so as is.
#pragma once

#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "pt_hip.h"
#include "pt_linalg.hpp"

#ifndef SEED
#define SEED 1
#endif

// rng.h:6-31 — the LCG the kernel runs per sample (reseeded by pt_sample_seed).
struct lcg {
    unsigned int state;
    const unsigned int a = 1664525;
    const unsigned int c = 1013904223;
    const unsigned long long m = 4294967296ull;
    lcg(unsigned int seed) : state(seed) {}
    unsigned int operator()() { return state = a * state + c; }
    float rand01() { return static_cast<float>((*this)()) / m; }
    void seed(unsigned int s) { state = s; }
    unsigned long long max() const { return m; }
    unsigned long long min() const { return 0; }
};
inline lcg rng(SEED);

struct AABB {
    vec3 lb = FLOAT_INF, rt = -FLOAT_INF;
    AABB() = default;
    AABB(const vec3& lb_, const vec3& rt_) : lb(lb_), rt(rt_) {}
    void merge(const AABB& o) {
        lb = component_min(lb, o.lb);
        rt = component_max(rt, o.rt);
    }
    void merge(const vec3& p) {
        lb = component_min(lb, p);
        rt = component_max(rt, p);
    }
    bool intersect_inv(const vec3& o, const vec3& inv) const {
        const vec3 t1 = (lb - o) * inv, t2 = (rt - o) * inv;
        const float tmax = std::min({std::max(t1.x, t2.x), std::max(t1.y, t2.y), std::max(t1.z, t2.z)});
        const float tmin = std::max({std::min(t1.x, t2.x), std::min(t1.y, t2.y), std::min(t1.z, t2.z)});
        return !(tmax < 0) && tmin <= tmax;
    }
    bool intersect(const vec3& o, const vec3& d) const { return intersect_inv(o, 1 / d); }
    bool is_valid() const { return lb.x <= rt.x && lb.y <= rt.y && lb.z <= rt.z; }
    float area() const {  // half the surface area
        if (!is_valid()) return 0;
        const vec3 e = rt - lb;
        return e.x * e.y + e.x * e.z + e.y * e.z;
    }
    friend std::ostream& operator<<(std::ostream& os, const AABB& b) { return os << "AABB: " << b.lb << " " << b.rt; }
};

// material.h:6-25. Host copies of the samplers (same draw order as the kernel).
inline vec3 hemisphere_sample(const vec3& /*ray_d*/, const vec3& normal) {
    const float u = rng.rand01();
    const float v = rng.rand01();
    const float theta = (float)((double)std::acos(2 * u - 1) - M_PI_2);
    const float phi = (float)(2 * M_PI * (double)v);
    const vec3 s(std::cos(theta) * std::cos(phi), std::cos(theta) * std::sin(phi), std::sin(theta));
    return s.dot(normal) < 0 ? -s : s;
}
inline vec3 specular_sample(const vec3& ray_d, const vec3& normal, float roughness) {
    const vec3 refl = ray_d - (2 * ray_d.dot(normal)) * normal;
    vec3 ret;
    do {
        const float jz = rng.rand01(), jy = rng.rand01(), jx = rng.rand01();
        ret = refl + (vec3(jx, jy, jz) - 0.5f) * roughness;
    } while (ret.dot(normal) < 0);
    return ret.normalize();
}

struct Material {
    enum Type : int32_t { EMIT = PT_MAT_EMIT, DIFFUSE = PT_MAT_DIFFUSE, SPECULAR = PT_MAT_SPECULAR } type;
    vec3 color;
    vec3 emit_color;
    float roughness;
    Material() = default;
    Material(Type t, const vec3& c, const vec3& e, float r) : type(t), color(c), emit_color(e), roughness(r) {}
    vec3 reflected_dir(const vec3& ray_d, const vec3& normal) const {
        switch (type) {
            case EMIT: return vec3(0, 0, 0);
            case SPECULAR: return specular_sample(ray_d, normal, roughness);
            default: return hemisphere_sample(ray_d, normal);
        }
    }
};
static_assert(sizeof(Material) == sizeof(pt_material), "Material must match pt_material");

struct Triangle {
    AABB aabb;
    vec3 centroid;
    vec3 v1, v2, v3;
    Material material;
    Triangle() = default;
    Triangle(const vec3& a, const vec3& b, const vec3& c, const Material& m) : centroid((a + b + c) / 3), v1(a), v2(b), v3(c), material(m) {
        aabb.merge(a);
        aabb.merge(b);
        aabb.merge(c);
    }
    bool intersect(const vec3& o, const vec3& d, float& t) const {
        const vec3 e1 = v2 - v1, e2 = v3 - v1, h = d.cross(e2);
        const float a = e1.dot(h);
        if (std::abs(a) < EPS) return false;
        const float f = 1 / a;
        const vec3 s = o - v1;
        const float u = f * s.dot(h);
        if (u < 0 || u > 1) return false;
        const vec3 q = s.cross(e1);
        const float v = f * d.dot(q);
        if (v < 0 || u + v > 1) return false;
        t = f * e2.dot(q);
        return t > 0;
    }
    vec3 normal(const vec3& ray_d, const vec3& /*p*/) const {
        const vec3 n = (v2 - v1).cross(v3 - v1).normalize();
        return n.dot(ray_d) < 0 ? n : -n;
    }
};

struct BVHNode {
    AABB aabb;
    int left, right;
    int tri_start, tri_end;
    BVHNode() = default;
    BVHNode(int l, int r, int s, int e) : left(l), right(r), tri_start(s), tri_end(e) {}
    bool is_leaf() const { return left == -1 && right == -1; }
};
static_assert(sizeof(BVHNode) == sizeof(pt_bvh_node), "BVHNode must match pt_bvh_node (40 B)");

struct BVH {
    bool built = false;
    std::vector<Triangle> triangles;
    std::vector<int> tri_idx;
    std::vector<BVHNode> nodes;

    BVH() = default;
    void add_triangle(const Triangle& t) {
        built = false;
        triangles.push_back(t);
    }
    size_t size() const { return triangles.size(); }
    bool empty() const { return triangles.empty(); }

    std::vector<float> packed_vertices() const {
        std::vector<float> v;
        v.reserve(9 * triangles.size());
        for (const Triangle& t : triangles)
            for (const vec3* p : {&t.v1, &t.v2, &t.v3}) v.insert(v.end(), {p->x, p->y, p->z});
        return v;
    }
    std::vector<pt_material> packed_materials() const {
        std::vector<pt_material> m(triangles.size());
        for (size_t i = 0; i < triangles.size(); i++) std::memcpy(&m[i], &triangles[i].material, sizeof(pt_material));
        return m;
    }

    // BVH::build (bvh.h:79-155) through libpt_hip.so's exact O(n log^2 n) builder.
    void build() {
        if (built) return;
        if (triangles.empty()) throw std::runtime_error("BVH::build: no triangles");
        const std::vector<float> v = packed_vertices();
        nodes.resize(2 * triangles.size() - 1);
        tri_idx.resize(triangles.size());
        const int n = pt_bvh_build((int32_t)triangles.size(), v.data(), reinterpret_cast<pt_bvh_node*>(nodes.data()),
                                   tri_idx.data());
        if (n < 0) throw std::runtime_error(std::string("BVH::build: ") + pt_last_error());
        nodes.resize(n);
        built = true;
    }

    // Wavefront OBJ + MTL import with the reference's material mapping (bvh.h:184-242):
    // illum 1 -> DIFFUSE(Kd), illum 2 -> EMIT(Ka), otherwise DIFFUSE(0.5). Polygons are
    // fan-triangulated; faces must reference a material (the reference indexes
    // materials[-1] otherwise).
    void load_obj(const std::string& filename, const std::string& mtl_path = "./") {
        std::ifstream in(filename);
        if (!in) throw std::runtime_error("TinyObjLoader: Cannot open file [" + filename + "]");
        std::vector<vec3> verts;
        std::map<std::string, Material> mats;
        const Material* cur = nullptr;
        std::string line;
        auto vtx = [&](const std::string& tok) {
            long i = std::stol(tok.substr(0, tok.find('/')));
            return verts.at(i > 0 ? (size_t)(i - 1) : (size_t)((long)verts.size() + i));
        };
        while (std::getline(in, line)) {
            std::istringstream ls(line);
            std::string tag;
            if (!(ls >> tag) || tag[0] == '#') continue;
            if (tag == "v") {
                double x, y, z;
                ls >> x >> y >> z;
                verts.emplace_back((float)x, (float)y, (float)z);
            } else if (tag == "mtllib") {
                std::string f;
                ls >> f;
                load_mtl(mtl_path + f, mats);
            } else if (tag == "usemtl") {
                std::string n;
                ls >> n;
                auto it = mats.find(n);
                if (it == mats.end()) throw std::runtime_error("TinyObjLoader: material '" + n + "' not found");
                cur = &it->second;
            } else if (tag == "f") {
                std::vector<std::string> f;
                for (std::string t; ls >> t;) f.push_back(t);
                if (f.size() < 3) continue;
                if (!cur) throw std::runtime_error("load_obj: face without material");
                for (size_t i = 1; i + 1 < f.size(); i++) add_triangle(Triangle(vtx(f[0]), vtx(f[i]), vtx(f[i + 1]), *cur));
            }
        }
    }

    void print(int node_idx = 0, int depth = 0, std::string dir = "root") const {
        if (node_idx == -1) return;
        std::cout << node_idx << ":\t";
        for (int i = 0; i < depth; i++) std::cout << " | ";
        if (depth > 0) std::cout << " +-";
        const BVHNode& n = nodes[node_idx];
        std::cout << n.aabb.lb << ' ' << n.aabb.rt << (n.is_leaf() ? " leaf, tri: " : " tri: ") << n.tri_start
                  << " -> " << n.tri_end << " (" << dir << ")\n";
        if (!n.is_leaf()) {
            print(n.left, depth + 1, "left");
            print(n.right, depth + 1, "right");
        }
    }

   private:
    static void load_mtl(const std::string& path, std::map<std::string, Material>& out) {
        std::ifstream in(path);
        if (!in) {
            std::cerr << "TinyObjLoader: Material file [ " << path << " ] not found.\n";
            return;
        }
        struct Raw { vec3 ka{0}, kd{0}; int illum = -1; };
        std::map<std::string, Raw> raw;
        std::string line, name;
        while (std::getline(in, line)) {
            std::istringstream ls(line);
            std::string tag;
            if (!(ls >> tag) || tag[0] == '#') continue;
            double a = 0, b = 0, c = 0;
            if (tag == "newmtl") { ls >> name; raw[name]; }
            else if (tag == "Ka") { ls >> a >> b >> c; raw[name].ka = vec3((float)a, (float)b, (float)c); }
            else if (tag == "Kd") { ls >> a >> b >> c; raw[name].kd = vec3((float)a, (float)b, (float)c); }
            else if (tag == "illum") { ls >> raw[name].illum; }
        }
        for (const auto& [n, r] : raw) {
            if (r.illum == 1) out[n] = Material(Material::DIFFUSE, r.kd, 0, 0);
            else if (r.illum == 2) out[n] = Material(Material::EMIT, 0, r.ka, 0);
            else {
                std::cerr << "Unknown material type with illum: " << r.illum << '\n'
                          << "Using default material: Diffuse(0.5)" << '\n';
                out[n] = Material(Material::DIFFUSE, 0.5, 0, 0);
            }
        }
    }
};
