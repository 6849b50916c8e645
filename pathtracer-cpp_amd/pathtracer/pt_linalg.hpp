// pt_linalg.hpp — math types of the drop-in API (reference: pathtracer/linalg.h).
// Same type names, members and operator set as the reference so user scene code
// compiles unchanged; everything is `inline` so the headers can be included from
// any number of translation units (the reference's are single-TU only).
#pragma once

#include <algorithm>
#include <array>
#include <cmath>
#include <functional>
#include <ostream>
#include <stdexcept>

#ifndef DEG2RAD
#define DEG2RAD M_PI / 180  // kept textually identical: `60 * DEG2RAD` == (60 * M_PI) / 180
#endif
#ifndef EPS
#define EPS 1e-6
#endif
#ifndef FLOAT_INF
#define FLOAT_INF 1e30
#endif

struct ivec2 {
    int x, y;
    ivec2() = default;
    ivec2(int v) : x(v), y(v) {}
    ivec2(int x_, int y_) : x(x_), y(y_) {}
    bool operator==(const ivec2& o) { return x == o.x && y == o.y; }
    bool operator!=(const ivec2& o) { return !(*this == o); }
    friend ivec2 component_max(const ivec2& a, const ivec2& b) { return {std::max(a.x, b.x), std::max(a.y, b.y)}; }
    friend ivec2 component_min(const ivec2& a, const ivec2& b) { return {std::min(a.x, b.x), std::min(a.y, b.y)}; }
};

struct vec2 {
    float x, y;
    vec2() = default;
    vec2(float v) : x(v), y(v) {}
    vec2(float x_, float y_) : x(x_), y(y_) {}
    vec2(ivec2 v) : x((float)v.x), y((float)v.y) {}
    bool operator==(const vec2& o) { return std::abs(x - o.x) < EPS && std::abs(y - o.y) < EPS; }
    bool operator!=(const vec2& o) { return !(*this == o); }
    friend std::ostream& operator<<(std::ostream& os, const vec2& v) { return os << "(" << v.x << ", " << v.y << ")"; }
};

#define PT_VEC2_BINOP(OP)                                                                          \
    inline vec2 operator OP(const vec2& a, const vec2& b) { return vec2(a.x OP b.x, a.y OP b.y); } \
    inline vec2 operator OP(const vec2& a, float s) { return vec2(a.x OP s, a.y OP s); }           \
    inline vec2 operator OP(float s, const vec2& a) { return vec2(s OP a.x, s OP a.y); }           \
    inline vec2& operator OP##=(vec2& a, const vec2& b) { a.x OP## = b.x; a.y OP## = b.y; return a; } \
    inline vec2& operator OP##=(vec2& a, float s) { a.x OP## = s; a.y OP## = s; return a; }
PT_VEC2_BINOP(+)
PT_VEC2_BINOP(-)
PT_VEC2_BINOP(*)
PT_VEC2_BINOP(/)
#undef PT_VEC2_BINOP

struct vec3 {
    float x, y, z;
    vec3() = default;
    vec3(float v) : x(v), y(v), z(v) {}
    vec3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}

    float& operator[](int i) {
        switch (i) {
            case 0: return x;
            case 1: return y;
            case 2: return z;
        }
        throw std::out_of_range("vec3 index out of range");
    }
    float operator[](int i) const { return const_cast<vec3&>(*this)[i]; }
    vec3 operator-() const { return vec3(-x, -y, -z); }
    bool operator==(const vec3& o) const {
        return std::abs(x - o.x) < EPS && std::abs(y - o.y) < EPS && std::abs(z - o.z) < EPS;
    }
    bool operator!=(const vec3& o) const { return !(*this == o); }

    // Operation order is part of the bit-parity contract (no FMA, as written).
    float dot(const vec3& o) const { return x * o.x + y * o.y + z * o.z; }
    vec3 cross(const vec3& o) const { return vec3(y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x); }
    float length() const { return std::sqrt(dot(*this)); }
    vec3 normalize() const {
        const float l = length();
        return vec3(x / l, y / l, z / l);
    }
    float angle(const vec3& o) const { return std::acos(dot(o) / (length() * o.length())); }
    float distance(const vec3& o) const { return vec3(x - o.x, y - o.y, z - o.z).length(); }
    vec3 reflect(const vec3& n) const {
        const float k = dot(n);
        return vec3(x - n.x * 2 * k, y - n.y * 2 * k, z - n.z * 2 * k);
    }
    float max() const { return std::max({x, y, z}); }
    float min() const { return std::min({x, y, z}); }
    vec3 apply(std::function<float(float)> f) const { return vec3(f(x), f(y), f(z)); }

    friend vec3 component_max(const vec3& a, const vec3& b) {
        return vec3(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z));
    }
    friend vec3 component_min(const vec3& a, const vec3& b) {
        return vec3(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z));
    }
    friend vec3 pow(const vec3& v, float p) { return vec3(std::pow(v.x, p), std::pow(v.y, p), std::pow(v.z, p)); }
    friend std::ostream& operator<<(std::ostream& os, const vec3& v) {
        return os << "(" << v.x << ", " << v.y << ", " << v.z << ")";
    }
};

#define PT_VEC3_BINOP(OP)                                                                                     \
    inline vec3 operator OP(const vec3& a, const vec3& b) { return vec3(a.x OP b.x, a.y OP b.y, a.z OP b.z); } \
    inline vec3 operator OP(const vec3& a, float s) { return vec3(a.x OP s, a.y OP s, a.z OP s); }             \
    inline vec3 operator OP(float s, const vec3& a) { return vec3(s OP a.x, s OP a.y, s OP a.z); }             \
    inline vec3& operator OP##=(vec3& a, const vec3& b) {                                                      \
        a.x OP## = b.x; a.y OP## = b.y; a.z OP## = b.z;                                                        \
        return a;                                                                                              \
    }                                                                                                          \
    inline vec3& operator OP##=(vec3& a, float s) {                                                            \
        a.x OP## = s; a.y OP## = s; a.z OP## = s;                                                              \
        return a;                                                                                              \
    }
PT_VEC3_BINOP(+)
PT_VEC3_BINOP(-)
PT_VEC3_BINOP(*)
PT_VEC3_BINOP(/)
#undef PT_VEC3_BINOP

namespace color {
inline const vec3 white(1, 1, 1), black(0, 0, 0), red(1, 0, 0), orange(1, 0.5, 0), yellow(1, 1, 0),
    green(0, 1, 0), blue(0, 0, 1), purple(0.5, 0, 0.5);
inline vec3 mix(const vec3& a, const vec3& b, float a_t = 0.5) { return a * (1 - a_t) + b * a_t; }
}  // namespace color

struct mat4 {
    std::array<std::array<float, 4>, 4> arr;
    mat4() = default;
    mat4(const mat4&) = default;
    mat4(float v) {
        for (auto& row : arr) row.fill(v);
    }
    std::array<float, 4>& operator[](size_t i) { return arr[i]; }
    const std::array<float, 4>& operator[](size_t i) const { return arr[i]; }
    vec3 transform_dir(const vec3& v) const {
        return vec3(v.dot({arr[0][0], arr[1][0], arr[2][0]}), v.dot({arr[0][1], arr[1][1], arr[2][1]}),
                    v.dot({arr[0][2], arr[1][2], arr[2][2]}));
    }
    friend std::ostream& operator<<(std::ostream& os, const mat4& m) {
        for (const auto& row : m.arr) os << "[" << row[0] << ", " << row[1] << ", " << row[2] << ", " << row[3] << "]\n";
        return os;
    }
};

inline float clamp(float x, float lo, float hi) { return std::max(lo, std::min(hi, x)); }
