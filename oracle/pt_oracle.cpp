// pt_oracle.cpp — CPU restatement of the reference hot path. TEST INFRASTRUCTURE.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library (oracle/liboracle.so), and only as the checker. The product
// (libpt_hip.so) never links or calls it.
//
// Parity pinned: tests/test_oracle_golden.py checks this restatement bit-for-bit
// against outputs of the unmodified reference compiled from /root/reference
// (oracle/ref/build_ref.sh -> oracle/_ref/pt_ref; fixtures in tests/golden/).
//
// Restates (reference file:line):
//   lcg                       rng.h:6-31       state = 1664525*state + 1013904223 (mod 2^32)
//   vec3 ops                  linalg.h:82-184  component order as written, no FMA
//   AABB::intersect_inv       aabb.h:20-29     std::min/max + min_element/max_element semantics
//   Triangle::intersect       triangle.h:25-44 Möller–Trumbore, |a| < EPS compared in double
//   Triangle::normal          triangle.h:45-49
//   hemisphere_sample         material.h:6-14
//   specular_sample           material.h:15-25
//   Material::reflected_dir   material.h:40-51
//   Camera ctor / get_ray     camera.h:33-73   (y jitter drawn first: g++ evaluates the
//                                               vec3(...) arguments right to left)
//   BVH::build                bvh.h:48-155
//   BVH::intersect            bvh.h:156-183    LIFO, right child popped first
//   trace                     render.h:36-61   recursive
//   gamma + quantisation      image.h:41-55, linalg.h:177-178,233-235 (oracle_rgb8; pinned to
//                                               the reference's PNG bytes, tests/test_rgb8.py)
//   render loop + /spp        render.h:80-97, image.h:37-40
// libm: acosf restates glibc 2.35 sysdeps/ieee754/flt-32/e_acosf.c (fdlibm);
// sincosf restates glibc 2.35 sysdeps/ieee754/flt-32/s_sincosf.c (ARM optimized
// routines, double-precision polynomial). tests/test_math.py checks both
// against the host glibc (exhaustively over the path's domain in the slow test).
#include <cmath>
#include <algorithm>
#include <thread>
#include <cstdint>
#include <cstring>
#include <deque>
#include <vector>

namespace orc {

// ---------------------------------------------------------------- libm
static inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

float acosf_(float x) {
    const float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    const float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f,
                pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f;
    const float qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f,
                qS4 = 7.7038154006e-02f;
    int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    auto P = [&](float z) { return z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5))))); };
    auto Q = [&](float z) { return 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4))); };
    if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;
        float z = x * x;
        float r = P(z) / Q(z);
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (hx < 0) {
        float z = (1.0f + x) * 0.5f;
        float p = P(z), q = Q(z);
        float s = std::sqrt(z);
        float r = p / q;
        float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    }
    float z = (1.0f - x) * 0.5f;
    float s = std::sqrt(z);
    float df = bitsf(fbits(s) & 0xfffff000u);
    float c = (z - df * df) / (s + df);
    float r = P(z) / Q(z);
    float w = r * s + c;
    return 2.0f * (df + w);
}

struct SinCosTab { double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; };
static const SinCosTab kSC[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, -0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
};
static inline uint32_t top12(float x) { return (fbits(x) >> 20) & 0x7ff; }

static void sincos_poly(double x, double x2, const SinCosTab* p, int n, float* sinp, float* cosp) {
    double x4 = x2 * x2, x3 = x2 * x;
    double c2 = p->c3 + x2 * p->c4, s1 = p->s2 + x2 * p->s3;
    if (n & 1) { float* t = sinp; sinp = cosp; cosp = t; }
    double c1 = p->c0 + x2 * p->c1, x5 = x3 * x2, x6 = x4 * x2;
    double s = x + x3 * p->s1, c = c1 + x4 * p->c2;
    *sinp = (float)(s + x5 * s1);
    *cosp = (float)(c + x6 * c2);
}

void sincosf_(float y, float* sinp, float* cosp) {
    double x = y;
    const SinCosTab* p = &kSC[0];
    if (top12(y) < top12((float)0x1.921FB54442D18p-1)) {
        if (top12(y) < top12(0x1p-12f)) { *sinp = y; *cosp = 1.0f; return; }
        sincos_poly(x, x * x, p, 0, sinp, cosp);
    } else if (top12(y) < top12(120.0f)) {
        double r = x * p->hpi_inv;
        int n = ((int32_t)r + 0x800000) >> 24;
        x = x - n * p->hpi;
        double s = p->sign[n & 3];
        if (n & 2) p = &kSC[1];
        sincos_poly(x * s, x * x, p, n, sinp, cosp);
    } else {
        // Outside the path's domain (|y| >= 120); fall back to the host libm.
        *sinp = std::sin(y);
        *cosp = std::cos(y);
    }
}

// ---------------------------------------------------------------- math
struct V3 {
    float x, y, z;
    V3() : x(0), y(0), z(0) {}
    V3(float v) : x(v), y(v), z(v) {}
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
};
static inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
static inline V3 operator/(float s, V3 a) { return {s / a.x, s / a.y, s / a.z}; }
static inline V3 operator-(V3 a, float s) { return {a.x - s, a.y - s, a.z - s}; }
static inline V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline V3 normalize(V3 a) { return a / std::sqrt(dot(a, a)); }
// std::max(a,b) / std::min(a,b)
static inline float smax(float a, float b) { return (a < b) ? b : a; }
static inline float smin(float a, float b) { return (b < a) ? b : a; }
// std::min({a,b,c}) / std::max({a,b,c}) via min_element / max_element
static inline float smin3(float a, float b, float c) { float r = a; if (b < r) r = b; if (c < r) r = c; return r; }
static inline float smax3(float a, float b, float c) { float r = a; if (r < b) r = b; if (r < c) r = c; return r; }

// ---------------------------------------------------------------- rng
struct Lcg {
    uint32_t state;
    uint32_t next() { state = 1664525u * state + 1013904223u; return state; }
    float rand01() { return (float)next() / 4294967296.0f; }
};

// ---------------------------------------------------------------- scene
enum { EMIT = 1, DIFFUSE = 2, SPECULAR = 3 };
struct Mat { int32_t type; V3 color, emit; float rough; };
struct Box {
    V3 lb{1e30f}, rt{-1e30f};
    void merge(const Box& o) {
        lb = V3(smin(lb.x, o.lb.x), smin(lb.y, o.lb.y), smin(lb.z, o.lb.z));
        rt = V3(smax(rt.x, o.rt.x), smax(rt.y, o.rt.y), smax(rt.z, o.rt.z));
    }
    void merge(V3 p) {
        lb = V3(smin(lb.x, p.x), smin(lb.y, p.y), smin(lb.z, p.z));
        rt = V3(smax(rt.x, p.x), smax(rt.y, p.y), smax(rt.z, p.z));
    }
    float half_area() const {
        if (!(lb.x <= rt.x && lb.y <= rt.y && lb.z <= rt.z)) return 0;
        V3 d = rt - lb;
        return d.x * d.y + d.x * d.z + d.y * d.z;
    }
    bool hit(V3 o, V3 inv) const {
        V3 t1 = (lb - o) * inv, t2 = (rt - o) * inv;
        float tmax = smin3(smax(t1.x, t2.x), smax(t1.y, t2.y), smax(t1.z, t2.z));
        float tmin = smax3(smin(t1.x, t2.x), smin(t1.y, t2.y), smin(t1.z, t2.z));
        if (tmax < 0) return false;
        return tmin <= tmax;
    }
};
struct Tri {
    V3 v1, v2, v3, centroid;
    Box box;
    Mat m;
    bool hit(V3 o, V3 d, float& t) const {
        V3 e1 = v2 - v1, e2 = v3 - v1;
        V3 h = cross(d, e2);
        float a = dot(e1, h);
        if ((double)std::fabs(a) < 1e-6) return false;
        float f = 1 / a;
        V3 s = o - v1;
        float u = f * dot(s, h);
        if (u < 0 || u > 1) return false;
        V3 q = cross(s, e1);
        float v = f * dot(d, q);
        if (v < 0 || u + v > 1) return false;
        t = f * dot(e2, q);
        return t > 0;
    }
    V3 normal(V3 d) const {
        V3 n = normalize(cross(v2 - v1, v3 - v1));
        return dot(n, d) < 0 ? n : neg(n);
    }
};
struct Node { Box box; int32_t left, right, start, end; };
static_assert(sizeof(Node) == 40, "node layout = reference BVHNode (40 B)");

struct Scene {
    std::vector<Tri> tris;
    std::vector<Node> nodes;
    std::vector<int32_t> idx;
    uint64_t rays = 0, node_visits = 0, tri_tests = 0, hits = 0;

    // BVH::intersect, bvh.h:156-183
    int intersect(V3 o, V3 d, float& t) {
        rays++;
        V3 inv = 1.0f / d;
        std::deque<int> st;
        st.push_back(0);
        int ret = -1;
        t = 1e30f;
        while (!st.empty()) {
            const Node& n = nodes[st.back()];
            st.pop_back();
            node_visits++;
            if (!n.box.hit(o, inv)) continue;
            if (n.left == -1 && n.right == -1) {
                for (int i = n.start; i <= n.end; i++) {
                    float tt;
                    tri_tests++;
                    if (tris[idx[i]].hit(o, d, tt) && tt < t) { t = tt; ret = idx[i]; }
                }
            } else {
                st.push_back(n.left);
                st.push_back(n.right);
            }
        }
        if (ret != -1) hits++;
        return ret;
    }
};

// BVH::build + find_best_axis, bvh.h:48-155
static void build(std::vector<Tri>& tris, std::vector<Node>& nodes, std::vector<int32_t>& idx) {
    const int n = (int)tris.size();
    idx.resize(n);
    for (int i = 0; i < n; i++) idx[i] = i;
    nodes.clear();
    nodes.reserve(2 * n);
    nodes.push_back(Node{Box{}, -1, -1, 0, n - 1});
    auto cen = [&](int i, int ax) { const V3& c = tris[idx[i]].centroid; return ax == 0 ? c.x : ax == 1 ? c.y : c.z; };
    std::deque<int> st;
    st.push_back(0);
    while (!st.empty()) {
        int ci = st.back();
        st.pop_back();
        for (int i = nodes[ci].start; i <= nodes[ci].end; i++) nodes[ci].box.merge(tris[idx[i]].box);
        const int s0 = nodes[ci].start, s1 = nodes[ci].end;
        int best_axis = -1;
        float split = 0, best = 1e30f;
        for (int ax = 0; ax < 3; ax++) {
            for (int i = s0; i <= s1; i++) {
                float pos = cen(i, ax);
                int lc = 0, rc = 0;
                Box lb, rb;
                for (int j = s0; j <= s1; j++) {
                    if (cen(j, ax) < pos) { lc++; lb.merge(tris[idx[j]].box); }
                    else { rc++; rb.merge(tris[idx[j]].box); }
                }
                if (lc == 0 || rc == 0) continue;
                float cost = lc * lb.half_area() + rc * rb.half_area();
                if (cost < best) { best = cost; best_axis = ax; split = pos; }
            }
        }
        int count = s1 - s0 + 1;
        float nosplit = count * nodes[ci].box.half_area();
        if (best_axis == -1 || best > nosplit) continue;
        int a = s0, b = s1, lcount = 0;
        while (a < b) {
            if (cen(a, best_axis) < split) { a++; lcount++; }
            else if (cen(b, best_axis) >= split) b--;
            else std::swap(idx[a], idx[b]);
        }
        if (lcount == 0 || lcount == count) continue;
        int L = (int)nodes.size();
        nodes.push_back(Node{Box{}, -1, -1, s0, s0 + lcount - 1});
        int R = (int)nodes.size();
        nodes.push_back(Node{Box{}, -1, -1, s0 + lcount, s1});
        nodes[ci].left = L;
        nodes[ci].right = R;
        st.push_back(L);
        st.push_back(R);
    }
}

struct Cam {
    V3 pos;
    int rx, ry;
    float vx, vy, cell, dist;
    float T[9];  // rows right, up, -forward
    void ray(Lcg& g, int w, int h, V3& o, V3& d) const {
        float jy = g.rand01();  // camera.h:64-65 under g++: second argument evaluated first
        float jx = g.rand01();
        V3 c((w + jx) * cell - vx / 2, (h + jy) * cell - vy / 2, -dist);
        d = normalize(V3(dot(c, V3(T[0], T[3], T[6])), dot(c, V3(T[1], T[4], T[7])),
                         dot(c, V3(T[2], T[5], T[8]))));
        o = pos;
    }
};

static V3 hemisphere(Lcg& g, V3 n) {
    float u = g.rand01();
    float v = g.rand01();
    float theta = (float)((double)acosf_(2 * u - 1) - 1.57079632679489661923);
    float phi = (float)(2 * 3.14159265358979323846 * (double)v);
    float st, ct, sp, cp;
    sincosf_(theta, &st, &ct);
    sincosf_(phi, &sp, &cp);
    V3 s(ct * cp, ct * sp, st);
    return dot(s, n) < 0 ? neg(s) : s;
}

static V3 specular(Lcg& g, V3 d, V3 n, float rough) {
    V3 refl = d - (2 * dot(d, n)) * n;
    V3 ret;
    do {
        float rz = g.rand01();  // vec3(rand01(), rand01(), rand01()) under g++: z, y, x
        float ry = g.rand01();
        float rx = g.rand01();
        V3 j = (V3(rx, ry, rz) - 0.5f) * rough;
        ret = refl + j;
    } while (dot(ret, n) < 0);
    return normalize(ret);
}

static V3 reflect_dir(Lcg& g, const Mat& m, V3 d, V3 n) {
    switch (m.type) {
        case EMIT: return V3(0, 0, 0);
        case SPECULAR: return specular(g, d, n, m.rough);
        default: return hemisphere(g, n);
    }
}

// trace, render.h:36-61
static V3 trace(Scene& sc, Lcg& g, V3 o, V3 d, int depth) {
    if (depth == 0) return V3(0.0f);
    float t;
    int hi = sc.intersect(o, d, t);
    if (hi == -1) return V3(0.0f);
    const Tri& tr = sc.tris[hi];
    if (tr.m.type == EMIT) return tr.m.emit;
    V3 p = o + d * t;
    V3 n = tr.normal(d);
    V3 nd = reflect_dir(g, tr.m, d, n);
    V3 no = p + n * 1e-4f;
    V3 rec = trace(sc, g, no, nd, depth - 1);
    float c = dot(n, nd);
    return tr.m.emit + ((2 * rec) * tr.m.color) * c;
}

}  // namespace orc

using namespace orc;

namespace {

uint64_t g_last[4];  // rays, node_visits, tri_tests, hits of the last oracle_render*
void keep_stats(const Scene& sc) {
    g_last[0] = sc.rays; g_last[1] = sc.node_visits; g_last[2] = sc.tri_tests; g_last[3] = sc.hits;
}

void load(Scene& sc, int ntris, const float* verts, const int32_t* mtype, const float* mvals,
          int nnodes, const void* nodes, const int32_t* tri_idx) {
    sc.tris.resize(ntris);
    for (int i = 0; i < ntris; i++) {
        Tri& t = sc.tris[i];
        const float* v = verts + 9 * i;
        t.v1 = V3(v[0], v[1], v[2]);
        t.v2 = V3(v[3], v[4], v[5]);
        t.v3 = V3(v[6], v[7], v[8]);
        t.centroid = (t.v1 + t.v2 + t.v3) / 3;  // triangle.h:17
        t.box = Box{};
        t.box.merge(t.v1);
        t.box.merge(t.v2);
        t.box.merge(t.v3);
        if (mtype) {
            const float* m = mvals + 7 * i;
            t.m.type = mtype[i];
            t.m.color = V3(m[0], m[1], m[2]);
            t.m.emit = V3(m[3], m[4], m[5]);
            t.m.rough = m[6];
        }
    }
    if (nodes) {
        sc.nodes.resize(nnodes);
        std::memcpy(sc.nodes.data(), nodes, sizeof(Node) * nnodes);
        sc.idx.assign(tri_idx, tri_idx + ntris);
    } else {
        build(sc.tris, sc.nodes, sc.idx);
    }
}

Cam make_cam(const float* c) {
    // c: pos[3], rx, ry, vx, vy, cell, dist, T[9] (as float; rx, ry stored as float)
    Cam k;
    k.pos = V3(c[0], c[1], c[2]);
    k.rx = (int)c[3];
    k.ry = (int)c[4];
    k.vx = c[5];
    k.vy = c[6];
    k.cell = c[7];
    k.dist = c[8];
    for (int i = 0; i < 9; i++) k.T[i] = c[9 + i];
    return k;
}

static inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
static inline uint32_t sample_seed(uint32_t p, uint32_t s, uint32_t seed) {
    return mix32(mix32(mix32(seed) ^ p) + s);
}

}  // namespace

extern "C" {

// Builds the BVH (bvh.h:79-155); nodes_out: 40-byte nodes (2n-1), idx_out: n ints.
int oracle_bvh_build(int ntris, const float* verts, void* nodes_out, int32_t* idx_out) {
    Scene sc;
    load(sc, ntris, verts, nullptr, nullptr, 0, nullptr, nullptr);
    std::memcpy(nodes_out, sc.nodes.data(), sizeof(Node) * sc.nodes.size());
    std::memcpy(idx_out, sc.idx.data(), 4 * sc.idx.size());
    return (int)sc.nodes.size();
}

// Camera ctor, camera.h:33-61. out: pos[3], rx, ry, vx, vy, cell, dist, T[9] (18 floats).
int oracle_camera(const float* pos, const float* fwd, const float* up, int rx, int ry, float fov,
                  float dist, float* out) {
    V3 P(pos[0], pos[1], pos[2]), F0(fwd[0], fwd[1], fwd[2]), U0(up[0], up[1], up[2]);
    V3 F = normalize(F0);
    V3 R = normalize(cross(F0, U0));
    V3 U = normalize(U0);
    if (std::fabs(dot(F, U)) > 0.999) return -1;
    float vx = 2 * dist * std::tan(fov / 2);
    float vy = 2 * dist * std::tan(fov / 2) * ry / rx;
    float cell = vx / rx;
    float c[18] = {P.x, P.y, P.z, (float)rx, (float)ry, vx, vy, cell, dist,
                   R.x, R.y, R.z, U.x, U.y, U.z, -F.x, -F.y, -F.z};
    std::memcpy(out, c, sizeof(c));
    return 0;
}

// Render rows [row_begin, row_end) of the image (render.h:80-97 with per-sample reseed).
// mvals: 7 floats per tri (color rgb, emit rgb, roughness). nodes == NULL -> build here.
// out: (row_end-row_begin) * W * 3 floats.
void oracle_render(int ntris, const float* verts, const int32_t* mtype, const float* mvals, int nnodes,
                   const void* nodes, const int32_t* tri_idx, const float* cam, int spp, int depth,
                   uint32_t seed, int row_begin, int row_end, float* out, uint64_t* rays) {
    Scene sc;
    load(sc, ntris, verts, mtype, mvals, nnodes, nodes, tri_idx);
    Cam k = make_cam(cam);
    Lcg g{0};
    size_t o = 0;
    for (int h = row_begin; h < row_end; h++)
        for (int w = 0; w < k.rx; w++) {
            V3 acc(0.0f);
            for (int s = 0; s < spp; s++) {
                g.state = sample_seed((uint32_t)(h * k.rx + w), (uint32_t)s, seed);
                V3 ro, rd;
                k.ray(g, w, h, ro, rd);
                acc = acc + trace(sc, g, ro, rd, depth);
            }
            acc = acc / (float)spp;
            out[o++] = acc.x;
            out[o++] = acc.y;
            out[o++] = acc.z;
        }
    keep_stats(sc);
    if (rays) *rays = sc.rays;
}

// Same, for an explicit list of pixels (w,h pairs); out: n * 3 floats.
void oracle_render_pixels(int ntris, const float* verts, const int32_t* mtype, const float* mvals,
                          int nnodes, const void* nodes, const int32_t* tri_idx, const float* cam,
                          int spp, int depth, uint32_t seed, const int32_t* px, int npx, float* out,
                          uint64_t* rays) {
    Scene sc;
    load(sc, ntris, verts, mtype, mvals, nnodes, nodes, tri_idx);
    Cam k = make_cam(cam);
    Lcg g{0};
    for (int i = 0; i < npx; i++) {
        int w = px[2 * i], h = px[2 * i + 1];
        V3 acc(0.0f);
        for (int s = 0; s < spp; s++) {
            g.state = sample_seed((uint32_t)(h * k.rx + w), (uint32_t)s, seed);
            V3 ro, rd;
            k.ray(g, w, h, ro, rd);
            acc = acc + trace(sc, g, ro, rd, depth);
        }
        acc = acc / (float)spp;
        out[3 * i] = acc.x;
        out[3 * i + 1] = acc.y;
        out[3 * i + 2] = acc.z;
    }
    keep_stats(sc);
    if (rays) *rays = sc.rays;
}

// Traversal counters of the last render: rays, node visits (pops), triangle tests, hits.
void oracle_last_stats(uint64_t* out4) { std::memcpy(out4, g_last, sizeof(g_last)); }

// ---- unit-level known-answer hooks ----
uint32_t oracle_sample_seed(uint32_t p, uint32_t s, uint32_t seed) { return sample_seed(p, s, seed); }
void oracle_lcg(uint32_t state, int n, uint32_t* out_states, float* out_rand01) {
    Lcg g{state};
    for (int i = 0; i < n; i++) {
        uint32_t st = g.state;
        out_states[i] = g.next();
        g.state = st;
        out_rand01[i] = g.rand01();
    }
}
float oracle_acosf(float x) { return acosf_(x); }
void oracle_sincosf_n(const float* x, int n, float* s, float* c) {
    for (int i = 0; i < n; i++) sincosf_(x[i], s + i, c + i);
}
void oracle_acosf_n(const float* x, int n, float* y) {
    for (int i = 0; i < n; i++) y[i] = acosf_(x[i]);
}
// Count mismatches vs the host libm over [lo, hi] (all floats); returns mismatches.
uint64_t oracle_libm_sweep(int which, float lo, float hi, uint64_t* tested) {
    uint64_t bad = 0, n = 0;
    for (int sg = 0; sg < 2; sg++)
        for (uint32_t u = 0;; u++) {
            float x = bitsf(u | (sg ? 0x80000000u : 0u));
            if (sg ? !(x >= lo) : !(x <= hi)) break;
            if (x < lo || x > hi) continue;
            n++;
            if (which == 0) {
                if (fbits(acosf_(x)) != fbits(::acosf(x))) bad++;
            } else {
                float s1, c1, s2, c2;
                sincosf_(x, &s1, &c1);
                ::sincosf(x, &s2, &c2);
                if (fbits(s1) != fbits(s2) || fbits(c1) != fbits(c2)) bad++;
            }
            if (u == 0x7f800000u) break;
        }
    if (tested) *tested = n;
    return bad;
}
// hemisphere_sample's first draw (material.h:8-9): x = 2 rand01 - 1 for EVERY 32-bit LCG
// state (rand01 = (float)state / 2^32). Returns how many x are off the grid k 2^-24 of
// [-1, 1] (0 makes the device's theta table, indexed by x 2^24 + 2^24, cover every x the
// path can draw); *at_one counts x == 1. Threads split the state range.
uint64_t oracle_theta_grid_check(uint64_t* at_one) {
    const int nt = 8;
    std::vector<uint64_t> bad(nt, 0), one(nt, 0);
    std::vector<std::thread> th;
    for (int k = 0; k < nt; k++)
        th.emplace_back([k, nt, &bad, &one] {
            const uint64_t lo = (1ull << 32) * k / nt, hi = (1ull << 32) * (k + 1) / nt;
            for (uint64_t st = lo; st < hi; st++) {  // next() is a bijection: st ranges over its outputs
                const float u = (float)(uint32_t)st / 4294967296.0f;  // Lcg::rand01 of that output
                const float x = 2.0f * u - 1.0f;
                const float y = x * 16777216.0f;
                if (!(x >= -1.0f && x <= 1.0f) || y != (float)(int64_t)y) bad[k]++;
                if (x == 1.0f) one[k]++;
            }
        });
    for (auto& t : th) t.join();
    uint64_t b = 0, o = 0;
    for (int k = 0; k < nt; k++) b += bad[k], o += one[k];
    if (at_one) *at_one = o;
    return b;
}
int oracle_tri_hit(const float* v, const float* o, const float* d, float* t) {
    Tri tr;
    tr.v1 = V3(v[0], v[1], v[2]);
    tr.v2 = V3(v[3], v[4], v[5]);
    tr.v3 = V3(v[6], v[7], v[8]);
    return tr.hit(V3(o[0], o[1], o[2]), V3(d[0], d[1], d[2]), *t) ? 1 : 0;
}
int oracle_slab(const float* lb, const float* rt, const float* o, const float* inv) {
    Box b;
    b.lb = V3(lb[0], lb[1], lb[2]);
    b.rt = V3(rt[0], rt[1], rt[2]);
    return b.hit(V3(o[0], o[1], o[2]), V3(inv[0], inv[1], inv[2])) ? 1 : 0;
}
// BRDF samples from a given LCG state; returns the state after the draws.
uint32_t oracle_brdf(uint32_t state, int type, float rough, const float* d, const float* n, float* out) {
    Lcg g{state};
    Mat m{type, V3(1.0f), V3(0.0f), rough};
    V3 r = reflect_dir(g, m, V3(d[0], d[1], d[2]), V3(n[0], n[1], n[2]));
    out[0] = r.x;
    out[1] = r.y;
    out[2] = r.z;
    return g.state;
}

// gamma_correct then save_png's quantisation of one value (image.h:41-55; vec3 pow,
// linalg.h:177-178; clamp, linalg.h:233-235).
static unsigned char q8(float p, float inv_gamma) {
    const float g = std::pow(p, inv_gamma);
    return static_cast<unsigned char>(std::max(0.0f, std::min(1.0f, g)) * 255);
}

// Image::gamma_correct + the byte buffer save_png encodes (image.h:41-55): rows top first.
void oracle_rgb8(const float* lin, int W, int H, float gamma, uint8_t* out) {
    const float inv = 1 / gamma;
    for (int h = 0; h < H; h++)
        for (int w = 0; w < W; w++)
            for (int c = 0; c < 3; c++)
                out[((size_t)h * W + w) * 3 + c] = q8(lin[((size_t)(H - h - 1) * W + w) * 3 + c], inv);
}

// The device quantiser's rule (pt_rgb8_kernel) on the float with bits `u`.
static unsigned char thr_rule(uint32_t u, const float* thr, int neg_mode) {
    float x;
    memcpy(&x, &u, 4);
    if (x != x) return 255;
    if (x < 0.0f && neg_mode != 2) return neg_mode == 0 ? 255 : 0;
    x = std::fabs(x);
    return (unsigned char)(std::upper_bound(thr, thr + 255, x) - thr);
}

// Counts the floats with bits lo, lo+step, ... < hi on which the threshold rule and q8
// disagree (nthreads workers).
uint64_t oracle_rgb8_sweep(float gamma, const float* thr255, int neg_mode, uint32_t lo, uint32_t hi, uint32_t step,
                           int nthreads) {
    const float inv = 1 / gamma;
    if (step == 0 || hi <= lo) return 0;
    const uint64_t n = ((uint64_t)hi - lo + step - 1) / step;
    nthreads = std::max(1, nthreads);
    std::vector<uint64_t> bad(nthreads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++)
        th.emplace_back([&, t]() {
            for (uint64_t i = (uint64_t)t; i < n; i += (uint64_t)nthreads) {
                const uint32_t u = lo + (uint32_t)(i * step);
                float x;
                memcpy(&x, &u, 4);
                if (q8(x, inv) != thr_rule(u, thr255, neg_mode)) bad[t]++;
            }
        });
    for (auto& x : th) x.join();
    uint64_t s = 0;
    for (uint64_t b : bad) s += b;
    return s;
}

}  // extern "C"
