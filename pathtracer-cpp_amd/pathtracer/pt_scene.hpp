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
    // bvh.h:184-242 through libpt_hip.so's tinyobjloader restatement (pt_obj_load):
    // same triangles, order, materials, stderr messages and exceptions.
    void load_obj(const std::string& filename, const std::string& mtl_path = "./") {
        pt_obj* obj = nullptr;
        if (pt_obj_load(filename.c_str(), mtl_path.c_str(), &obj) != PT_OK)
            throw std::runtime_error(pt_last_error());
        const std::string warn = pt_obj_warnings(obj);
        if (!warn.empty()) std::cerr << "TinyObjLoader: " << warn << '\n';
        const size_t n = (size_t)pt_obj_num_tris(obj);
        std::vector<float> v(9 * n);
        std::vector<Material> mats(n);
        std::vector<int32_t> illum(n);
        static_assert(sizeof(Material) == sizeof(pt_material), "Material layout");
        pt_obj_triangles(obj, v.data(), reinterpret_cast<pt_material*>(mats.data()), illum.data());
        pt_obj_free(obj);
        for (size_t i = 0; i < n; i++) {
            if (illum[i] != 1 && illum[i] != 2) {
                std::cerr << "Unknown material type with illum: " << illum[i] << '\n';
                std::cerr << "Using default material: Diffuse(0.5)" << '\n';
            }
            const float* p = &v[9 * i];
            add_triangle(Triangle(vec3(p[0], p[1], p[2]), vec3(p[3], p[4], p[5]), vec3(p[6], p[7], p[8]), mats[i]));
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
};
