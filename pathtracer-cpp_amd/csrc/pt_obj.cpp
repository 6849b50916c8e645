// pt_obj.cpp — OBJ/MTL ingestion for BVH::load_obj (bvh.h:184-242), host side.
//
// The reference reads meshes through its vendored tinyobjloader v2
// (pathtracer/tiny_obj_loader.h, ObjReaderConfig defaults: triangulate with the
// built-in method) and maps materials in bvh.h:216-238. This file restates the
// parts that decide which triangles come out, in which order, with which bits and
// materials (line numbers into tiny_obj_loader.h):
//   lines             safeGetline 764-796: "\n", "\r\n" and "\r" end a line; leading
//                     " \t" skipped; '#' comments
//   numbers           tryParseDouble 893-1027: decimal digits accumulated in a double
//                     (fraction digits scaled by 10^-k), exponent applied as
//                     ldexp(m * pow(5, e), e); parseReal 1029-1060: default 0 when a
//                     field is missing or malformed, narrowed to float
//   face indices      parseTriple 1155-1207 / fixIndex 815-846: 1-based, negative =
//                     relative to the elements read so far, 0 is an error for vertices
//   triangulation     exportGroupsToShape 1447-1930, run when a face group is flushed
//                     (usemtl change, g, o, end of file) against the vertices read by
//                     then: triangles as written; quads split on the shorter diagonal
//                     (|v2-v0|^2 < |v3-v1|^2 ? 012,023 : 013,123); larger polygons by
//                     ear clipping in the plane of the first non-degenerate corner,
//                     with pnpoly (1406-1414) rejecting ears that contain a vertex
//   materials         usemtl 2723-2745 (a face's material is the one current when it
//                     is read), mtllib 2747-2838, MaterialFileReader 2400-2455
//                     (':'-separated search path, JoinPath 1999-2011), LoadMtl
//                     2013-2396 (newmtl / Ka / Kd / illum / map_Kd's 0.6 default; the
//                     first definition of a name wins; the last material is flushed
//                     even without a name)
//   mapping           bvh.h:216-238: illum 1 -> DIFFUSE(Kd), 2 -> EMIT(Ka), anything
//                     else -> DIFFUSE(0.5); the first three corners of each triangle
// The reference indexes materials[-1] for a face without a material and reads past
// the vertex array for an index beyond it (undefined behaviour): both are errors here.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "pt_hip.h"
#include "pt_internal.h"

using pt::set_error;

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t'; }
inline bool is_digit(char c) { return (unsigned)(c - '0') < 10u; }
inline bool is_eol(char c) { return c == '\r' || c == '\n' || c == '\0'; }

// One line as safeGetline delivers it; false at the end of the stream.
bool next_line(std::istream& is, std::string& t) {
    t.clear();
    std::streambuf* sb = is.rdbuf();
    int c = sb->sbumpc();
    if (c == EOF) return false;
    for (;; c = sb->sbumpc()) {
        if (c == EOF || c == '\n') return true;
        if (c == '\r') {
            if (sb->sgetc() == '\n') sb->sbumpc();
            return true;
        }
        t += (char)c;
    }
}

// tryParseDouble over [s, e): false when no number starts at s.
bool parse_double(const char* s, const char* e, double* out) {
    if (s >= e) return false;
    const char* p = s;
    bool neg = false, dot_first = false;
    if (*p == '+' || *p == '-') {
        neg = *p == '-';
        p++;
        dot_first = p != e && *p == '.';
    } else if (*p == '.') {
        dot_first = true;
    } else if (!is_digit(*p)) {
        return false;
    }
    double m = 0.0;
    int exp10 = 0;
    if (!dot_first) {
        int n = 0;
        for (; p != e && is_digit(*p); p++, n++) m = m * 10 + (int)(*p - '0');
        if (n == 0) return false;
    }
    if (p != e && *p == '.') {
        static const double kScale[8] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
        p++;
        for (int k = 1; p != e && is_digit(*p); p++, k++)
            m += (int)(*p - '0') * (k < 8 ? kScale[k] : std::pow(10.0, -k));
    }
    if (p != e && (*p == 'e' || *p == 'E')) {
        p++;
        bool eneg = false;
        if (p != e && (*p == '+' || *p == '-')) {
            eneg = *p == '-';
            p++;
        } else if (!is_digit(*p)) {
            return false;
        }
        int n = 0;
        for (; p != e && is_digit(*p); p++, n++) {
            if (exp10 > 2147483647 / 10) return false;
            exp10 = exp10 * 10 + (int)(*p - '0');
        }
        if (n == 0) return false;
        if (eneg) exp10 = -exp10;
    }
    *out = (neg ? -1 : 1) * (exp10 ? std::ldexp(m * std::pow(5.0, exp10), exp10) : m);
    return true;
}

// parseReal: the next whitespace-delimited field as a float, `dflt` if it is not a number.
float parse_real(const char** tok, double dflt = 0.0) {
    *tok += strspn(*tok, " \t");
    const char* end = *tok + strcspn(*tok, " \t\r");
    double v = dflt;
    parse_double(*tok, end, &v);
    *tok = end;
    return (float)v;
}

std::string parse_word(const char** tok) {
    *tok += strspn(*tok, " \t");
    const size_t n = strcspn(*tok, " \t\r");
    std::string s(*tok, n);
    *tok += n;
    return s;
}

bool fix_index(int idx, int n, int* out, bool allow_zero) {
    if (idx > 0) {
        *out = idx - 1;
        return true;
    }
    if (idx == 0) {
        *out = -1;
        return allow_zero;
    }
    *out = n + idx;
    return *out >= 0;
}

// parseTriple: "v", "v/t", "v//n" or "v/t/n"; only the vertex index is kept.
bool parse_corner(const char** tok, int nv, int nn, int nt, int* v) {
    int unused;
    if (!fix_index(atoi(*tok), nv, v, false)) return false;
    *tok += strcspn(*tok, "/ \t\r");
    if ((*tok)[0] != '/') return true;
    (*tok)++;
    if ((*tok)[0] == '/') {
        (*tok)++;
        if (!fix_index(atoi(*tok), nn, &unused, true)) return false;
        *tok += strcspn(*tok, "/ \t\r");
        return true;
    }
    if (!fix_index(atoi(*tok), nt, &unused, true)) return false;
    *tok += strcspn(*tok, "/ \t\r");
    if ((*tok)[0] != '/') return true;
    (*tok)++;
    if (!fix_index(atoi(*tok), nn, &unused, true)) return false;
    *tok += strcspn(*tok, "/ \t\r");
    return true;
}

struct Mtl {
    std::string name;
    float ka[3] = {0, 0, 0}, kd[3] = {0, 0, 0};
    int illum = 0;
};

// LoadMtl: appends the file's materials; a name already in `index` keeps its first slot.
void load_mtl(std::istream& in, std::vector<Mtl>& mats, std::map<std::string, int>& index) {
    Mtl cur;
    bool has_kd = false;  // set by any Kd of the file, never reset (LoadMtl)
    std::string line;
    while (in.peek() != EOF && next_line(in, line)) {
        line = line.substr(0, line.find_last_not_of(" \t") + 1);
        if (!line.empty() && line.back() == '\n') line.pop_back();
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty()) continue;
        const char* t = line.c_str() + strspn(line.c_str(), " \t");
        if (t[0] == '\0' || t[0] == '#') continue;
        if (!strncmp(t, "newmtl", 6) && is_space(t[6])) {
            if (!cur.name.empty()) {
                index.insert({cur.name, (int)mats.size()});
                mats.push_back(cur);
            }
            cur = Mtl();
            t += 7;
            cur.name = parse_word(&t);
        } else if (t[0] == 'K' && (t[1] == 'a' || t[1] == 'd') && is_space(t[2])) {
            float* dst = t[1] == 'a' ? cur.ka : cur.kd;
            if (t[1] == 'd') has_kd = true;
            t += 2;
            for (int k = 0; k < 3; k++) dst[k] = parse_real(&t);
        } else if (!strncmp(t, "illum", 5) && is_space(t[5])) {
            t += 6;
            t += strspn(t, " \t");
            cur.illum = atoi(t);
        } else if (!strncmp(t, "map_Kd", 6) && is_space(t[6])) {
            if (!has_kd) cur.kd[0] = cur.kd[1] = cur.kd[2] = 0.6f;
        }
    }
    index.insert({cur.name, (int)mats.size()});
    mats.push_back(cur);
}

struct Face {
    std::vector<int> v;  // vertex indices (0-based)
    int mat;
};

std::string join_path(const std::string& dir, const std::string& f) {
    if (dir.empty()) return f;
    return dir.back() == '/' ? dir + f : dir + "/" + f;
}

}  // namespace

struct pt_obj {
    std::vector<float> verts;      // 9 per triangle
    std::vector<pt_material> mats; // per triangle
    std::vector<int32_t> illum;    // per triangle: the MTL illum value behind it
    std::string warnings;
};

namespace {

struct Loader {
    std::vector<float> v;  // x, y, z per vertex
    int nn = 0, nt = 0;
    std::vector<Mtl> mats;
    std::map<std::string, int> index;
    std::set<std::string> mtl_files;
    std::string search_path;
    std::vector<Face> pending;
    std::vector<std::pair<std::vector<int>, int>> tris;  // corners, material id
    std::string warn;

    float coord(size_t vi, size_t axis) const { return v[vi * 3 + axis]; }
    bool valid(size_t vi) const { return 3 * vi + 2 < v.size(); }

    void emit(int a, int b, int c, int mat) { tris.push_back({{a, b, c}, mat}); }

    // exportGroupsToShape for the faces read since the last flush.
    void flush() {
        for (const Face& f : pending) {
            const size_t n = f.v.size();
            if (n < 3) {
                warn += "Degenerated face found\n.";
                continue;
            }
            if (n == 3) {
                emit(f.v[0], f.v[1], f.v[2], f.mat);
            } else if (n == 4) {
                quad(f);
            } else {
                ear_clip(f);
            }
        }
        pending.clear();
    }

    void quad(const Face& f) {
        const size_t i0 = f.v[0], i1 = f.v[1], i2 = f.v[2], i3 = f.v[3];
        if (!valid(i0) || !valid(i1) || !valid(i2) || !valid(i3)) {
            warn += "Face with invalid vertex index found.\n";
            return;
        }
        const float e02x = coord(i2, 0) - coord(i0, 0), e02y = coord(i2, 1) - coord(i0, 1),
                    e02z = coord(i2, 2) - coord(i0, 2);
        const float e13x = coord(i3, 0) - coord(i1, 0), e13y = coord(i3, 1) - coord(i1, 1),
                    e13z = coord(i3, 2) - coord(i1, 2);
        const float sqr02 = e02x * e02x + e02y * e02y + e02z * e02z;
        const float sqr13 = e13x * e13x + e13y * e13y + e13z * e13z;
        if (sqr02 < sqr13) {
            emit(f.v[0], f.v[1], f.v[2], f.mat);
            emit(f.v[0], f.v[2], f.v[3], f.mat);
        } else {
            emit(f.v[0], f.v[1], f.v[3], f.mat);
            emit(f.v[1], f.v[2], f.v[3], f.mat);
        }
    }

    static bool point_in_tri(const float* xs, const float* ys, float tx, float ty) {
        bool c = false;
        for (int i = 0, j = 2; i < 3; j = i++)
            if (((ys[i] > ty) != (ys[j] > ty)) && (tx < (xs[j] - xs[i]) * (ty - ys[i]) / (ys[j] - ys[i]) + xs[i]))
                c = !c;
        return c;
    }

    void ear_clip(const Face& f) {
        const size_t n0 = f.v.size();
        // projection plane: drop the axis of the first corner's largest cross component
        size_t ax0 = 1, ax1 = 2;
        for (size_t k = 0; k < n0; k++) {
            const size_t a = f.v[k % n0], b = f.v[(k + 1) % n0], c = f.v[(k + 2) % n0];
            if (!valid(a) || !valid(b) || !valid(c)) continue;
            const float e0x = coord(b, 0) - coord(a, 0), e0y = coord(b, 1) - coord(a, 1),
                        e0z = coord(b, 2) - coord(a, 2);
            const float e1x = coord(c, 0) - coord(b, 0), e1y = coord(c, 1) - coord(b, 1),
                        e1z = coord(c, 2) - coord(b, 2);
            const float cx = std::fabs(e0y * e1z - e0z * e1y), cy = std::fabs(e0z * e1x - e0x * e1z),
                        cz = std::fabs(e0x * e1y - e0y * e1x);
            if (cx > FLT_EPSILON || cy > FLT_EPSILON || cz > FLT_EPSILON) {
                if (!(cx > cy && cx > cz)) {
                    ax0 = 0;
                    if (cz > cx && cz > cy) ax1 = 1;
                }
                break;
            }
        }
        std::vector<int> rem = f.v;
        size_t guess = 0, budget = n0, last_n = n0;
        while (rem.size() > 3 && budget > 0) {
            const size_t n = rem.size();
            if (guess >= n) guess -= n;
            if (last_n != n) {
                last_n = n;
                budget = n;
            } else {
                budget--;
            }
            int ind[3];
            float xs[3], ys[3];
            for (int k = 0; k < 3; k++) {
                ind[k] = rem[(guess + k) % n];
                const size_t vi = ind[k];
                const bool ok = vi * 3 + ax0 < v.size() && vi * 3 + ax1 < v.size();
                xs[k] = ok ? v[vi * 3 + ax0] : 0.0f;
                ys[k] = ok ? v[vi * 3 + ax1] : 0.0f;
            }
            const float e0x = xs[1] - xs[0], e0y = ys[1] - ys[0], e1x = xs[2] - xs[1], e1y = ys[2] - ys[1];
            const float cross = e0x * e1y - e0y * e1x;
            const float area = (xs[0] * ys[1] - ys[0] * xs[1]) * 0.5f;
            if (cross * area < 0.0f) {  // reflex corner
                guess++;
                continue;
            }
            bool inside = false;
            for (size_t o = 3; o < n && !inside; o++) {
                const size_t vi = rem[(guess + o) % n];
                if (vi * 3 + ax0 >= v.size() || vi * 3 + ax1 >= v.size()) continue;
                inside = point_in_tri(xs, ys, v[vi * 3 + ax0], v[vi * 3 + ax1]);
            }
            if (inside) {
                guess++;
                continue;
            }
            emit(ind[0], ind[1], ind[2], f.mat);
            rem.erase(rem.begin() + (long)((guess + 1) % n));
        }
        if (rem.size() == 3) emit(rem[0], rem[1], rem[2], f.mat);
    }

    bool read_mtl_file(const std::string& name) {
        if (search_path.empty()) {
            std::ifstream in(name);
            if (!in) return false;
            load_mtl(in, mats, index);
            return true;
        }
        std::istringstream paths(search_path);
        std::string dir;
        while (std::getline(paths, dir, ':')) {
            std::ifstream in(join_path(dir, name));
            if (in) {
                load_mtl(in, mats, index);
                return true;
            }
        }
        warn += "Material file [ " + name + " ] not found in a path : " + search_path + "\n";
        return false;
    }

    void mtllib(const char* t) {
        std::vector<std::string> names;  // SplitString(' ', '\\')
        std::string cur;
        bool esc = false;
        for (const char* p = t; *p; p++) {
            if (esc) {
                esc = false;
            } else if (*p == '\\') {
                esc = true;
                continue;
            } else if (*p == ' ') {
                if (!cur.empty()) names.push_back(cur);
                cur.clear();
                continue;
            }
            cur += *p;
        }
        names.push_back(cur);
        bool found = false;
        for (const std::string& nm : names) {
            if (mtl_files.count(nm)) {
                found = true;
                continue;
            }
            if (read_mtl_file(nm)) {
                found = true;
                mtl_files.insert(nm);
                break;
            }
        }
        if (!found) warn += "Failed to load material file(s). Use default material.\n";
    }

    int parse(std::istream& in) {
        int material = -1;
        std::string line;
        size_t line_no = 0;
        while (in.peek() != EOF && next_line(in, line)) {
            line_no++;
            if (!line.empty() && line.back() == '\n') line.pop_back();
            if (!line.empty() && line.back() == '\r') line.pop_back();
            if (line.empty()) continue;
            const char* t = line.c_str() + strspn(line.c_str(), " \t");
            if (t[0] == '\0' || t[0] == '#') continue;
            if (t[0] == 'v' && is_space(t[1])) {
                t += 2;
                for (int k = 0; k < 3; k++) v.push_back(parse_real(&t));
            } else if (t[0] == 'v' && (t[1] == 'n' || t[1] == 't') && is_space(t[2])) {
                (t[1] == 'n' ? nn : nt)++;
            } else if ((t[0] == 'f' || t[0] == 'l' || t[0] == 'p') && is_space(t[1])) {
                const char kind = t[0];
                t += 2;
                if (kind == 'f') t += strspn(t, " \t");
                Face f{{}, material};
                while (!is_eol(t[0])) {
                    int vi;
                    if (!parse_corner(&t, (int)(v.size() / 3), nn, nt, &vi))
                        return set_error(PT_E_ARG, "TinyObjLoader: Failed to parse `%c' line (e.g. a zero value for "
                                         "vertex index). Line %zu.", kind, line_no);
                    f.v.push_back(vi);
                    t += strspn(t, " \t\r");
                }
                if (kind == 'f') pending.push_back(std::move(f));
            } else if (!strncmp(t, "usemtl", 6)) {
                t += 6;
                const std::string name = parse_word(&t);
                auto it = index.find(name);
                int id = -1;
                if (it != index.end()) id = it->second;
                else warn += "material [ '" + name + "' ] not found in .mtl\n";
                if (id != material) {
                    flush();
                    material = id;
                }
            } else if (!strncmp(t, "mtllib", 6) && is_space(t[6])) {
                mtllib(t + 7);
            } else if ((t[0] == 'g' || t[0] == 'o') && is_space(t[1])) {
                flush();
            }
        }
        flush();
        return PT_OK;
    }
};

}  // namespace

extern "C" {

int pt_obj_load(const char* filename, const char* mtl_search_path, pt_obj** out) {
    if (!filename || !out) return set_error(PT_E_ARG, "pt_obj_load: NULL argument");
    *out = nullptr;
    std::ifstream in(filename);
    if (!in) return set_error(PT_E_IO, "TinyObjLoader: Cannot open file [%s]", filename);
    Loader L;
    if (mtl_search_path && *mtl_search_path) {
        L.search_path = mtl_search_path;
    } else {  // ObjReader::ParseFromFile: the OBJ file's directory
        const std::string f(filename);
        const size_t pos = f.find_last_of("/\\");
        if (pos != std::string::npos) L.search_path = f.substr(0, pos);
    }
    int rc = L.parse(in);
    if (rc) return rc;
    const size_t nverts = L.v.size() / 3;
    pt_obj* o = new pt_obj();
    o->warnings = L.warn;
    o->verts.reserve(9 * L.tris.size());
    for (const auto& tr : L.tris) {
        if (tr.second < 0) {
            delete o;
            return set_error(PT_E_ARG,
                             "load_obj: a face has no material (no usemtl, or an unknown name); the reference "
                             "would index materials[-1] (bvh.h:217-218)");
        }
        for (int k = 0; k < 3; k++) {
            const size_t vi = (size_t)tr.first[k];
            if (vi >= nverts) {
                delete o;
                return set_error(PT_E_ARG, "load_obj: vertex index %zu beyond the %zu vertices", vi + 1, nverts);
            }
            for (int a = 0; a < 3; a++) o->verts.push_back(L.v[3 * vi + a]);
        }
        const Mtl& m = L.mats[tr.second];
        pt_material pm;
        memset(&pm, 0, sizeof(pm));
        if (m.illum == 1) {  // Material(DIFFUSE, Kd, 0, 0)
            pm.type = PT_MAT_DIFFUSE;
            memcpy(pm.color, m.kd, sizeof(pm.color));
        } else if (m.illum == 2) {  // Material(EMIT, 0, Ka, 0)
            pm.type = PT_MAT_EMIT;
            memcpy(pm.emit, m.ka, sizeof(pm.emit));
        } else {  // Material(DIFFUSE, 0.5, 0, 0)
            pm.type = PT_MAT_DIFFUSE;
            pm.color[0] = pm.color[1] = pm.color[2] = 0.5f;
        }
        o->mats.push_back(pm);
        o->illum.push_back(m.illum);
    }
    *out = o;
    return PT_OK;
}

int32_t pt_obj_num_tris(const pt_obj* o) { return o ? (int32_t)o->mats.size() : 0; }

int pt_obj_triangles(const pt_obj* o, float* verts, pt_material* mats, int32_t* illum) {
    if (!o) return set_error(PT_E_ARG, "pt_obj_triangles: NULL object");
    if (verts && !o->verts.empty()) memcpy(verts, o->verts.data(), o->verts.size() * sizeof(float));
    if (mats && !o->mats.empty()) memcpy(mats, o->mats.data(), o->mats.size() * sizeof(pt_material));
    if (illum && !o->illum.empty()) memcpy(illum, o->illum.data(), o->illum.size() * sizeof(int32_t));
    return PT_OK;
}

const char* pt_obj_warnings(const pt_obj* o) { return o ? o->warnings.c_str() : ""; }

void pt_obj_free(pt_obj* o) { delete o; }

}  // extern "C"
