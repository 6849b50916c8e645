// pt_host.cpp — host half of libpt_hip.so: errors, BVH construction, camera
// setup, scene validation/packing, 8-bit post-process and PNG output.
//
// Built with -ffp-contract=off (no FMA on the host either), so every float
// expression here rounds exactly like the reference's g++ -O3 x86-64 build.
#include <math.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "pt_internal.h"
#include "pt_math.h"

namespace pt {

static thread_local std::string g_err;

int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

const char* hook_env(const char* name) {
    static const bool enabled = [] {
        const char* g = getenv("PT_TEST_HOOKS");
        return g && strcmp(g, "1") == 0;
    }();
    return enabled ? getenv(name) : nullptr;
}

namespace {

// AABB in the reference's semantics (aabb.h:6-47): empty box = {+1e30, -1e30}.
struct Box {
    v3 lb{1e30f, 1e30f, 1e30f};
    v3 rt{-1e30f, -1e30f, -1e30f};
    void grow(const v3& p) {
        lb = v3{std_min(lb.x, p.x), std_min(lb.y, p.y), std_min(lb.z, p.z)};
        rt = v3{std_max(rt.x, p.x), std_max(rt.y, p.y), std_max(rt.z, p.z)};
    }
    void grow(const Box& b) {
        lb = v3{std_min(lb.x, b.lb.x), std_min(lb.y, b.lb.y), std_min(lb.z, b.lb.z)};
        rt = v3{std_max(rt.x, b.rt.x), std_max(rt.y, b.rt.y), std_max(rt.z, b.rt.z)};
    }
    // AABB::area: half surface area, 0 for an invalid box (aabb.h:34-39)
    float half_area() const {
        if (!(lb.x <= rt.x && lb.y <= rt.y && lb.z <= rt.z)) return 0.0f;
        v3 d = sub(rt, lb);
        return d.x * d.y + d.x * d.z + d.y * d.z;
    }
};

struct TriKey {
    float c[3];  // centroid (v1+v2+v3)/3, triangle.h:17
    Box box;     // triangle.h:19-22
};

// Split search equivalent to BVH::find_best_axis (bvh.h:48-78) in O(m log m) per axis.
// The reference tries every (axis, position i) candidate, pos = centroid[axis] of the
// triangle at position i, left = {centroid < pos}, and keeps the FIRST candidate (in
// axis-major, position order) with the smallest cost below FLOAT_INF. All candidates
// with one value share one partition and cost, so per distinct value only the
// smallest position matters; boxes are min/max merges, independent of merge order.
struct Split {
    int axis = -1;
    int pos_index = 0;  // position of the winning candidate (tie-break key)
    float value = 0.0f;
    float cost = 1e30f;
};

// A triangle of a node's range in one axis's sweep: centroid value, position, box.
struct SweepItem {
    float v;
    int pos;
    Box box;
};

// The best split of one axis (the reference's candidates of that axis, in position order).
void axis_split(const std::vector<TriKey>& kord, int s0, int s1, int ax,
                Split& best, std::vector<SweepItem>& items, std::vector<Box>& suffix, std::vector<uint64_t>& rk,
                std::vector<uint64_t>& rk2) {
    const int m = s1 - s0 + 1;
    suffix.resize(m + 1);
    items.resize(m);
    // sorted by (centroid, position): the reference's candidate order, with each item's
    // box carried along so that the two sweeps below read memory in order. Large ranges:
    // a stable LSD radix sort of order-preserving centroid keys (positions are generated
    // in increasing order, so stability is the position tie-break; -0 is keyed as +0,
    // since the reference compares them equal).
    if (m < 1024) {
        for (int k = 0; k < m; k++) {
            const TriKey& t = kord[s0 + k];
            items[k] = SweepItem{t.c[ax], s0 + k, t.box};
        }
        std::sort(items.begin(), items.end(),
                  [](const SweepItem& a, const SweepItem& b) { return a.v < b.v || (a.v == b.v && a.pos < b.pos); });
    } else {
        rk.resize(m);
        rk2.resize(m);
        for (int k = 0; k < m; k++) {
            const float v = kord[s0 + k].c[ax];
            uint32_t u = v == 0.0f ? 0u : f2u(v);
            u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
            rk[k] = ((uint64_t)u << 32) | (uint32_t)k;
        }
        for (int shift = 32; shift < 64; shift += 8) {  // the key's four bytes, low to high
            uint32_t cnt[257] = {0};
            for (int k = 0; k < m; k++) cnt[((rk[k] >> shift) & 255u) + 1]++;
            for (int b = 0; b < 256; b++) cnt[b + 1] += cnt[b];
            for (int k = 0; k < m; k++) rk2[cnt[(rk[k] >> shift) & 255u]++] = rk[k];
            rk.swap(rk2);
        }
        for (int k = 0; k < m; k++) {
            const int j = (int)(uint32_t)rk[k];
            const TriKey& t = kord[s0 + j];
            items[k] = SweepItem{t.c[ax], s0 + j, t.box};
        }
    }
    suffix[m] = Box{};
    for (int k = m - 1; k >= 0; k--) {
        suffix[k] = suffix[k + 1];
        suffix[k].grow(items[k].box);
    }
    Box prefix;
    for (int k = 0; k < m; k++) {
        const float v = items[k].v;
        const bool first_of_value = (k == 0) || (items[k - 1].v != v);
        if (first_of_value && k > 0) {
            const int lc = k, rc = m - k;
            const float cost = lc * prefix.half_area() + rc * suffix[k].half_area();
            const int pi = items[k].pos;  // smallest position holding value v
            if (cost < best.cost || (cost == best.cost && best.axis == ax && pi < best.pos_index)) {
                best.cost = cost;
                best.axis = ax;
                best.pos_index = pi;
                best.value = v;
            }
        }
        prefix.grow(items[k].box);
    }
}

// Scratch of one axis sweep.
struct SplitScratch {
    std::vector<SweepItem> items;
    std::vector<Box> suffix;
    std::vector<uint64_t> rk, rk2;
};

// Ranges this large sweep their three axes on three threads (the reference's SAH peels
// a few triangles off a large node at a time, so a chain of large nodes is the critical
// path of the build, whatever the parallelism across subtrees). Helper threads count
// against kMaxBuildThreads like subtree threads (declared below).
constexpr int kParallelAxes = 8192;
constexpr int kMaxBuildThreads = 16;  // a GPU box's CPU share (hardware_concurrency counts the whole host)
static std::atomic<int> g_build_threads{0};

// A builder thread, if one of the kMaxBuildThreads slots is free and the system gives
// one; else nothing (the caller runs the work itself). Joined (and its slot returned) on
// destruction, so an exception on the calling thread unwinds safely.
struct Helper {
    std::thread t;
    template <typename F>
    explicit Helper(F&& f) {
        if (g_build_threads.fetch_add(1) < kMaxBuildThreads) {
            try {
                t = std::thread(std::forward<F>(f));
                return;
            } catch (const std::system_error&) {
            }
        }
        g_build_threads.fetch_sub(1);
    }
    bool running() const { return t.joinable(); }
    ~Helper() {
        if (t.joinable()) {
            t.join();
            g_build_threads.fetch_sub(1);
        }
    }
};

Split best_split(const std::vector<TriKey>& kord, int s0, int s1, SplitScratch (&sc)[3]) {
    Split per[3];
    bool done = false;
    if (s1 - s0 + 1 >= kParallelAxes) {
        auto sweep = [&](int ax) {
            axis_split(kord, s0, s1, ax, per[ax], sc[ax].items, sc[ax].suffix, sc[ax].rk, sc[ax].rk2);
        };
        Helper h1([&] { sweep(1); }), h2([&] { sweep(2); });
        sweep(0);
        if (!h1.running()) sweep(1);
        if (!h2.running()) sweep(2);
        done = true;  // h2, h1 joined here
    }
    if (!done) {
        for (int ax = 0; ax < 3; ax++) {
            per[ax] = Split{};
            axis_split(kord, s0, s1, ax, per[ax], sc[0].items, sc[0].suffix, sc[0].rk, sc[0].rk2);
        }
    }
    // axis-major scan order: a later axis wins only with a strictly smaller cost
    Split best = per[0];
    for (int ax = 1; ax < 3; ax++)
        if (per[ax].axis == ax && per[ax].cost < best.cost) best = per[ax];
    return best;
}

// ---- the same split search over per-axis lists sorted once (round 6, default builder).
// Each axis keeps the elements (triangle ids) of every node's position range sorted by
// centroid, as one contiguous segment; a partition splits the segments stably by the
// elements' new positions, so no node sorts again. Ties between equal centroids are in no
// particular order: the search only needs each value's least position (the reference's first
// candidate of that value), taken as a minimum over the tie group, and the prefix / suffix
// boxes are order-independent merges (min / max: only the sign of a zero bound can depend on
// the order, and no cost or comparison sees it). Same splits, same tree, bit for bit.
struct SortedBuild {
    const std::vector<TriKey>& key;  // by triangle id (immutable)
    std::vector<int32_t>& idx;       // position -> triangle id (the reference's tri_idx)
    std::vector<int32_t> where;      // triangle id -> position
    std::vector<int32_t> sorted[3];  // per axis: triangle ids, each node's segment sorted by centroid
    SortedBuild(const std::vector<TriKey>& k, std::vector<int32_t>& i) : key(k), idx(i) {}
};

struct SortedScratch {
    std::vector<Box> suffix;
    std::vector<int32_t> tmp;
};

void sorted_axis_split(const SortedBuild& B, int s0, int s1, int ax, Split& best, std::vector<Box>& suffix) {
    const int m = s1 - s0 + 1;
    const int32_t* L = B.sorted[ax].data() + s0;
    const TriKey* key = B.key.data();
    suffix.resize(m + 1);
    suffix[m] = Box{};
    for (int k = m - 1; k >= 0; k--) {
        suffix[k] = suffix[k + 1];
        suffix[k].grow(key[L[k]].box);
    }
    Box prefix;
    for (int k = 0; k < m;) {
        const float v = key[L[k]].c[ax];
        int g = k, pmin = INT32_MAX;
        float vmin = v;
        for (; g < m && key[L[g]].c[ax] == v; g++) {  // the value's tie group [k, g)
            const int pos = B.where[L[g]];
            if (pos < pmin) {
                pmin = pos;
                vmin = key[L[g]].c[ax];
            }
        }
        if (k > 0) {
            const int lc = k, rc = m - k;
            const float cost = lc * prefix.half_area() + rc * suffix[k].half_area();
            if (cost < best.cost || (cost == best.cost && best.axis == ax && pmin < best.pos_index)) {
                best.cost = cost;
                best.axis = ax;
                best.pos_index = pmin;
                best.value = vmin;
            }
        }
        for (; k < g; k++) prefix.grow(key[L[k]].box);
    }
}

Split sorted_best_split(const SortedBuild& B, int s0, int s1, SortedScratch (&sc)[3]) {
    Split per[3];
    if (s1 - s0 + 1 >= kParallelAxes) {
        Helper h1([&] { sorted_axis_split(B, s0, s1, 1, per[1], sc[1].suffix); });
        Helper h2([&] { sorted_axis_split(B, s0, s1, 2, per[2], sc[2].suffix); });
        sorted_axis_split(B, s0, s1, 0, per[0], sc[0].suffix);
        if (!h1.running()) sorted_axis_split(B, s0, s1, 1, per[1], sc[0].suffix);
        if (!h2.running()) sorted_axis_split(B, s0, s1, 2, per[2], sc[0].suffix);
    } else {
        for (int ax = 0; ax < 3; ax++) sorted_axis_split(B, s0, s1, ax, per[ax], sc[0].suffix);
    }
    Split best = per[0];
    for (int ax = 1; ax < 3; ax++)
        if (per[ax].axis == ax && per[ax].cost < best.cost) best = per[ax];
    return best;
}

// Every axis's list sorted by centroid (LSD radix sort of order-preserving keys, -0 keyed as
// +0: the reference compares them equal).
void sort_axis(SortedBuild& B, int ax) {
    const int n = (int)B.key.size();
    std::vector<uint64_t> rk(n), rk2(n);
    for (int e = 0; e < n; e++) {
        const float v = B.key[e].c[ax];
        uint32_t u = v == 0.0f ? 0u : f2u(v);
        u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        rk[e] = ((uint64_t)u << 32) | (uint32_t)e;
    }
    for (int shift = 32; shift < 64; shift += 8) {
        uint32_t cnt[257] = {0};
        for (int k = 0; k < n; k++) cnt[((rk[k] >> shift) & 255u) + 1]++;
        for (int b = 0; b < 256; b++) cnt[b + 1] += cnt[b];
        for (int k = 0; k < n; k++) rk2[cnt[(rk[k] >> shift) & 255u]++] = rk[k];
        rk.swap(rk2);
    }
    B.sorted[ax].resize(n);
    for (int k = 0; k < n; k++) B.sorted[ax][k] = (int32_t)(uint32_t)rk[k];
}

}  // namespace

// One axis of a wide node's quantisation: origin O = the node's least child lb (a
// float), scale 2^e with (hi - O) / 2^e <= qmax - 1 and 2^e >= ulp(max |coordinate|) / 2^8,
// so (c - O) / 2^e computed in double is within 2^-19 of its real value. Child planes
// lo = floor(x - 2^-16), hi = ceil(x + 2^-16) (clamped to [0, qmax]) then satisfy
// O + lo 2^e <= lb and O + hi 2^e >= rt as REAL numbers: the quantised box contains the
// reference's box (DESIGN.md §3.7 needs nothing more). qmax: 255 for byte planes, 2047
// for half planes (every integer up to 2048 is an exact binary16 value).
struct AxisQuant {
    float origin;
    int e;
    double qmax;
};

static AxisQuant axis_quant(float lo, float hi, int qmax) {
    const double ext = (double)hi - (double)lo;
    const float mag = std::max(fabsf(lo), fabsf(hi));
    const double span = qmax - 1;
    int e_ulp = -100;
    if (mag > 0.0f) e_ulp = std::max(-100, ilogbf(mag) - 23 - 8);
    int e = ext > 0.0 ? (int)ceil(log2(ext / span)) : -100;
    e = std::max(e, e_ulp);
    while (ldexp(ext, -e) > span) e++;
    return AxisQuant{lo, e, (double)qmax};
}

static uint32_t quant_lo(float c, const AxisQuant& q) {
    const double x = ldexp((double)c - (double)q.origin, -q.e);
    return (uint32_t)std::max(0.0, std::min(q.qmax, floor(x - 0x1p-16)));
}
static uint32_t quant_hi(float c, const AxisQuant& q) {
    const double x = ldexp((double)c - (double)q.origin, -q.e);
    return (uint32_t)std::max(0.0, std::min(q.qmax, ceil(x + 0x1p-16)));
}

// binary16 bits of an integer 0 <= n < 2048 (exact)
static uint16_t half_of_int(uint32_t n) {
    if (n == 0) return 0;
    int e = 31 - __builtin_clz(n);
    return (uint16_t)(((uint32_t)(e + 15) << 10) | ((n << (10 - e)) & 0x3ffu));
}
static uint32_t int_of_half(uint16_t h) {
    if (h == 0) return 0;
    const int e = (h >> 10) - 15;
    const uint32_t m = (h & 0x3ffu) | 0x400u;
    return e >= 10 ? m << (e - 10) : m >> (10 - e);
}

// Plane value j (lo or hi) of axis a of a quantised wide node (byte or binary16 planes).
static uint32_t wide_plane(const uint32_t* u, int W, bool f16, int a, int j, bool hi) {
    if (f16) {
        const uint16_t* h = reinterpret_cast<const uint16_t*>(u + 8) + (size_t)2 * W * a;
        return int_of_half(h[(hi ? W : 0) + j]);
    }
    const uint8_t* b = reinterpret_cast<const uint8_t*>(u + 8) + (size_t)4 * W * a;
    return b[(hi ? W : 0) + j];
}

// Collapse the binary tree into W-wide nodes with quantised child boxes (pt_internal.h
// "wide"/"wtris"). A node's children start as its binary children; the inner child with
// the largest surface area is replaced by its two children until W are collected. Any
// collapse tests exactly the reference's triangles: a conservative box
// never skips a leaf whose exact box passes, and a triangle hit only counts once the
// leaf's exact box passes too. Returns false (no wide path) for inputs the format
// cannot hold: > 255 triangles under one node's leaves, > 2^24 nodes, coordinates of
// magnitude >= 2^64.
// SAH-optimal collapse of the binary tree into W-wide nodes (the dynamic programme of
// Ylitie, Karras & Laine 2017, without its leaf merging): the cost of a wide node is the
// surface area of its box (the probability that a line through the scene visits it), and
// D[n][i] is the least total cost of representing binary node n's subtree by at most i
// child slots, either as one slot (a leaf, or a wide node of its own) or split between
// its two children. choice[n][i] = 0 takes n as a slot, k > 0 gives k slots to the left
// child; choice[n][0] is the split when n itself is a wide node. The exact test does not
// depend on the grouping, only the number of node visits does.
// Threads for the scene packing (pack_scene): PT_PACK_THREADS (test hook) or up to 8. The
// output does not depend on it (tests/test_capi.py: pt_debug_pack_hash at 1 and 8 threads).
static int pack_threads() {
    const char* e = hook_env("PT_PACK_THREADS");
    if (e && *e) return std::max(1, std::min(64, atoi(e)));
    return (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
}

// fn(begin, end) over [0, n) in chunks taken from a shared counter by up to `threads` threads,
// the calling thread one of them (alone when no thread can be started).
template <typename F>
static void parallel_chunks(size_t n, size_t chunk, int threads, F&& fn) {
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (;;) {
            const size_t b = next.fetch_add(chunk);
            if (b >= n) return;
            fn(b, std::min(n, b + chunk));
        }
    };
    std::vector<std::thread> ts;
    for (int t = 1; t < threads && (size_t)t * chunk < n; t++) {
        try {
            ts.emplace_back(work);
        } catch (const std::system_error&) {
            break;
        }
    }
    work();
    for (std::thread& t : ts) t.join();
}

struct WideCollapse {
    std::vector<std::array<uint8_t, 9>> choice;
};

// SAH-optimal collapse of the binary tree into W-wide nodes (cost tables D[n][i]: node n's
// subtree given i child slots), children before parents. Subtrees below the first levels are
// independent, so they run on `threads` threads and the levels above them after.
static WideCollapse sah_collapse(const pt_scene* s, int W, int threads) {
    const int nn = s->num_nodes;
    std::unique_ptr<std::array<double, 9>[]> D(new std::array<double, 9>[nn]);  // every reachable node written
    WideCollapse wc;
    wc.choice.resize(nn);
    auto area = [&](int n) {
        const pt_bvh_node& nd = s->nodes[n];
        const double x = (double)nd.rt[0] - nd.lb[0], y = (double)nd.rt[1] - nd.lb[1], z = (double)nd.rt[2] - nd.lb[2];
        return x * y + y * z + z * x;
    };
    auto is_leaf = [&](int n) { return s->nodes[n].left == -1 && s->nodes[n].right == -1; };
    auto cost = [&](int n) {
        const pt_bvh_node& nd = s->nodes[n];
        std::array<uint8_t, 9>& ch = wc.choice[n];
        ch.fill(0);
        if (is_leaf(n)) {
            for (int i = 0; i <= W; i++) D[n][i] = 0.0;
            return;
        }
        const auto &L = D[nd.left], &R = D[nd.right];
        double open = INFINITY;
        for (int k = 1; k < W; k++)
            if (L[k] + R[W - k] < open) {
                open = L[k] + R[W - k];
                ch[0] = (uint8_t)k;
            }
        const double inner = area(n) + open;  // n as a wide node of its own
        D[n][0] = INFINITY;
        D[n][1] = inner;
        for (int i = 2; i <= W; i++) {
            D[n][i] = inner;
            for (int k = 1; k < i; k++)
                if (L[k] + R[i - k] < D[n][i]) {
                    D[n][i] = L[k] + R[i - k];
                    ch[i] = (uint8_t)k;
                }
        }
    };
    // children before parents over the subtree of `root` (post-order by a reversed pre-order)
    auto subtree = [&](int root, std::vector<int32_t>& order) {
        order.clear();
        order.push_back(root);
        for (size_t i = 0; i < order.size(); i++) {
            const int n = order[i];
            if (!is_leaf(n)) {
                order.push_back(s->nodes[n].left);
                order.push_back(s->nodes[n].right);
            }
        }
        for (size_t o = order.size(); o-- > 0;) cost(order[o]);
    };
    // the first levels (breadth first) until 8 subtrees per thread hang below them
    std::vector<int32_t> upper, frontier{0};
    while (threads > 1 && nn > 4096 && (int)frontier.size() < 8 * threads) {
        std::vector<int32_t> next;
        bool grew = false;
        for (int n : frontier) {
            if (is_leaf(n)) {
                next.push_back(n);
                continue;
            }
            upper.push_back(n);
            next.push_back(s->nodes[n].left);
            next.push_back(s->nodes[n].right);
            grew = true;
        }
        frontier.swap(next);
        if (!grew) break;
    }
    parallel_chunks(frontier.size(), 1, threads, [&](size_t b, size_t e) {
        std::vector<int32_t> order;
        for (size_t i = b; i < e; i++) subtree(frontier[i], order);
    });
    for (size_t i = upper.size(); i-- > 0;) cost(upper[i]);  // BFS order reversed: children first
    return wc;
}

// The child slots of wide node n under a collapse: binary node m given i slots.
static void wide_slots(const pt_scene* s, const WideCollapse& wc, int m, int i, std::vector<int32_t>& out) {
    const uint8_t k = wc.choice[m][i];
    if (k == 0 || (s->nodes[m].left == -1 && s->nodes[m].right == -1)) {
        out.push_back(m);
        return;
    }
    wide_slots(s, wc, s->nodes[m].left, k, out);
    wide_slots(s, wc, s->nodes[m].right, i - k, out);
}

// The header words of a wide node in either layout (pt_internal.h).
struct WideHdr {
    int ni, nl;
    uint32_t child_base, leaf_base;
    const uint8_t* ends;  // cumulative triangle end offset of leaf k (byte k)
};
static WideHdr wide_hdr(const uint32_t* u, int fmt) {
    if (fmt == kWideF32)
        return WideHdr{(int)((u[0] >> 24) & 15u), (int)(u[0] >> 28), u[0] & 0xffffffu, u[1],
                       reinterpret_cast<const uint8_t*>(u + 2)};
    return WideHdr{(int)((u[3] >> 24) & 15u), (int)(u[3] >> 28), u[4], u[5], reinterpret_cast<const uint8_t*>(u + 6)};
}

static bool build_wide(const pt_scene* s, const std::vector<int32_t>& rank_pos, int W, int fmt, PackedScene& out,
                       std::vector<int32_t>* slot_nodes = nullptr) {
    const bool f16 = fmt == kWideF16, f32 = fmt == kWideF32;
    const int qmax = f16 ? 2047 : 255;
    const int U = 4 * kWideNodeU4(W, fmt), QW = W / 4;  // uint32 per node, uint32 per byte array
    float span[3] = {0.0f, 0.0f, 0.0f};  // kWideF32: max |plane| per axis
    auto is_leaf = [&](int n) { return s->nodes[n].left == -1 && s->nodes[n].right == -1; };
    auto area = [&](int n) {
        const pt_bvh_node& nd = s->nodes[n];
        const double x = (double)nd.rt[0] - nd.lb[0], y = (double)nd.rt[1] - nd.lb[1], z = (double)nd.rt[2] - nd.lb[2];
        return x * y + y * z + z * x;
    };
    for (size_t i = 0; i < 9 * (size_t)s->num_tris; i++)
        if (!(fabsf(s->verts[i]) < 0x1p64f)) return false;
    const int threads = pack_threads();
    // Phase 1, serial and breadth first: each wide node's child slots (inner children, then
    // the non-empty leaves), the BFS index of its first inner child and the wide-leaf-order
    // index of its first triangle. Phase 2 fills the nodes and triangle records from these
    // on `threads` threads (round 6: the per-node loop was most of config 4's scene setup).
    std::vector<int32_t> queue{0}, level{0}, slot_of;  // slot_of: W entries per node, -1 past its slots
    std::vector<uint8_t> n_inner, n_leaf;
    std::vector<uint32_t> child_base, leaf_base;
    const size_t max_wide = (size_t)std::max<int32_t>(1, s->num_nodes / 2);
    queue.reserve((size_t)s->num_nodes);
    level.reserve((size_t)s->num_nodes);
    slot_of.reserve((size_t)W * max_wide);
    n_inner.reserve(max_wide);
    n_leaf.reserve(max_wide);
    child_base.reserve(max_wide);
    leaf_base.reserve(max_wide);
    std::vector<int32_t> kids, inner, leaves;  // per node, reused
    kids.reserve(2 * (size_t)W);
    inner.reserve(W);
    leaves.reserve(W);
    int max_level = 0;
    bool single = true;
    uint32_t ntri = 0;  // triangles so far in wide-leaf order
    // SAH-optimal grouping by default; PT_WIDE_COLLAPSE=greedy opens the inner child with
    // the largest surface area until W children are collected (round-2 trees)
    const char* ce = hook_env("PT_WIDE_COLLAPSE");
    const bool greedy = ce && strcmp(ce, "greedy") == 0;
    WideCollapse wc;
    if (!greedy) wc = sah_collapse(s, W, threads);
    for (size_t w = 0; w < queue.size(); w++) {
        const pt_bvh_node& b = s->nodes[queue[w]];
        kids.clear();
        if (greedy) {
            kids = {b.left, b.right};
        } else {
            wide_slots(s, wc, b.left, wc.choice[queue[w]][0], kids);
            wide_slots(s, wc, b.right, W - wc.choice[queue[w]][0], kids);
        }
        while (greedy && (int)kids.size() < W) {
            int best = -1;
            double ba = -1.0;
            for (size_t i = 0; i < kids.size(); i++)
                if (!is_leaf(kids[i]) && area(kids[i]) > ba) {
                    ba = area(kids[i]);
                    best = (int)i;
                }
            if (best < 0) break;
            const int k = kids[best];
            kids[best] = s->nodes[k].left;
            kids.push_back(s->nodes[k].right);
        }
        inner.clear();
        leaves.clear();
        for (int k : kids) {
            if (!is_leaf(k)) inner.push_back(k);
            else if (s->nodes[k].tri_start <= s->nodes[k].tri_end) leaves.push_back(k);  // empty leaves test nothing
        }
        const int ni = (int)inner.size(), nl = (int)leaves.size();
        if (ni + nl > W) return false;
        n_inner.push_back((uint8_t)ni);
        n_leaf.push_back((uint8_t)nl);
        child_base.push_back((uint32_t)queue.size());  // inner children are the next BFS nodes
        leaf_base.push_back(ntri);
        for (int j = 0; j < W; j++) {
            const int32_t sl = j < ni ? inner[j] : j < ni + nl ? leaves[j - ni] : -1;
            slot_of.push_back(sl);
            if (slot_nodes) slot_nodes->push_back(sl);
        }
        for (int k : inner) {
            queue.push_back(k);
            level.push_back(level[w] + 1);
            max_level = std::max(max_level, level[w] + 1);
        }
        int run = 0;
        for (int k : leaves) {
            const pt_bvh_node& nd = s->nodes[k];
            if (nd.tri_end != nd.tri_start) single = false;
            run += nd.tri_end - nd.tri_start + 1;
        }
        if (run > 255) return false;  // leaf ends are bytes
        ntri += (uint32_t)run;
        if (queue.size() >= (1u << 24)) return false;
    }
    const size_t nw = queue.size();
    std::vector<uint32_t> buf(nw * (size_t)U, 0u);
    std::vector<f4> wt(4 * (size_t)ntri);
    std::vector<int32_t> wt_tri(ntri);  // per wide-order triangle: its position in tri_idx (for the compact records)
    std::atomic<bool> planes_ok{true};
    std::atomic<bool> tri_boxes{true};  // every single-triangle leaf's box is its triangle's AABB (compact records)
    std::mutex span_mu;
    parallel_chunks(nw, 256, threads, [&](size_t w0, size_t w1) {
        float sp[3] = {0.0f, 0.0f, 0.0f};
        bool boxes = true;
        for (size_t w = w0; w < w1; w++) {
            uint32_t* u = buf.data() + w * (size_t)U;
            const int ni = n_inner[w], nl = n_leaf[w], ns = ni + nl;
            const int32_t* slots = slot_of.data() + w * (size_t)W;
            AxisQuant aq[3];
            if (f32) {
                // header {child_base | ni << 24 | nl << 28, leaf_base, ends}; the planes are the
                // reference's own boxes, bit for bit (an empty slot: lo = +inf, hi = -inf, which
                // fails every ray's test)
                u[0] = child_base[w] | (uint32_t)ni << 24 | (uint32_t)nl << 28;
                u[1] = leaf_base[w];
                for (int a = 0; a < 3; a++)
                    for (int j = 0; j < W; j++) {
                        const bool used = j < ns;
                        const float lo = used ? s->nodes[slots[j]].lb[a] : INFINITY;
                        const float hi = used ? s->nodes[slots[j]].rt[a] : -INFINITY;
                        // the per-ray margin's bound needs finite planes below 2^64
                        if (used && !(fabsf(lo) < 0x1p64f && fabsf(hi) < 0x1p64f)) planes_ok = false;
                        u[4 + 2 * W * a + j] = f2u(lo);
                        u[4 + 2 * W * a + W + j] = f2u(hi);
                        if (used) sp[a] = std::max(sp[a], std::max(fabsf(lo), fabsf(hi)));
                    }
            } else {
                for (int a = 0; a < 3; a++) {
                    float lo = 1e30f, hi = -1e30f;
                    for (int j = 0; j < ns; j++) {
                        lo = std::min(lo, s->nodes[slots[j]].lb[a]);
                        hi = std::max(hi, s->nodes[slots[j]].rt[a]);
                    }
                    if (ns == 0) lo = hi = 0.0f;
                    aq[a] = axis_quant(lo, hi, qmax);
                    u[a] = f2u(aq[a].origin);
                }
                u[3] = (uint32_t)(aq[0].e + 128) | (uint32_t)(aq[1].e + 128) << 8 | (uint32_t)(aq[2].e + 128) << 16 |
                       (uint32_t)ni << 24 | (uint32_t)nl << 28;
                u[4] = child_base[w];
                u[5] = leaf_base[w];
                // axis a's plane block from word 8: byte planes lo[W] hi[W] hi[W] lo[W] (QW words
                // each; a ray reads (entry, exit) = (lo, hi) at its start for inv >= 0 and (hi, lo)
                // 2 QW words in for inv < 0, one aligned load with no per-child select), or half
                // planes lo[W] hi[W] (a ray reads its entry run at lo or hi and its exit run at the
                // other, two aligned loads)
                auto put = [&](int a, int j, uint32_t lo, uint32_t hi) {
                    if (f16) {
                        uint16_t* h = reinterpret_cast<uint16_t*>(u + 8) + (size_t)2 * W * a;
                        h[j] = half_of_int(lo);
                        h[W + j] = half_of_int(hi);
                        return;
                    }
                    uint8_t* b = reinterpret_cast<uint8_t*>(u + 8) + (size_t)16 * QW * a;
                    b[j] = (uint8_t)lo;
                    b[4 * QW + j] = (uint8_t)hi;
                    b[8 * QW + j] = (uint8_t)hi;
                    b[12 * QW + j] = (uint8_t)lo;
                };
                for (int j = 0; j < W; j++)
                    for (int a = 0; a < 3; a++) put(a, j, (uint32_t)qmax, 0);  // empty slot
                for (int j = 0; j < ns; j++) {
                    const pt_bvh_node& nd = s->nodes[slots[j]];
                    for (int a = 0; a < 3; a++) put(a, j, quant_lo(nd.lb[a], aq[a]), quant_hi(nd.rt[a], aq[a]));
                }
            }
            uint8_t* ends = reinterpret_cast<uint8_t*>(u + (f32 ? 2 : 6));
            uint32_t t = leaf_base[w];
            int run = 0;
            for (int k = 0; k < nl; k++) {
                const pt_bvh_node& nd = s->nodes[slots[ni + k]];
                for (int i = nd.tri_start; i <= nd.tri_end; i++, t++, run++) {
                    const float* v = s->verts + 9 * (size_t)s->tri_idx[i];
                    // the compact records rebuild the leaf box from the vertices: only exact for
                    // boxes equal to that AABB (== : -0 and +0 count as equal, NaN never does)
                    for (int a = 0; a < 3 && boxes; a++) {
                        const float lo = std::min(std::min(v[a], v[3 + a]), v[6 + a]);
                        const float hi = std::max(std::max(v[a], v[3 + a]), v[6 + a]);
                        if (!(nd.lb[a] == lo && nd.rt[a] == hi)) boxes = false;
                    }
                    const v3 v1{v[0], v[1], v[2]}, v2{v[3], v[4], v[5]}, v3_{v[6], v[7], v[8]};
                    const v3 e1 = sub(v2, v1), e2 = sub(v3_, v1);
                    f4* r = &wt[4 * (size_t)t];
                    r[0] = f4{v1.x, v1.y, v1.z, e1.x};
                    r[1] = f4{e1.y, e1.z, e2.x, e2.y};
                    r[2] = f4{e2.z, u2f((uint32_t)rank_pos[i]), nd.lb[0], nd.lb[1]};
                    r[3] = f4{nd.lb[2], nd.rt[0], nd.rt[1], nd.rt[2]};
                    wt_tri[t] = i;
                }
                ends[k] = (uint8_t)run;
            }
        }
        if (!boxes) tri_boxes = false;
        std::lock_guard<std::mutex> lk(span_mu);
        for (int a = 0; a < 3; a++) span[a] = std::max(span[a], sp[a]);
    });
    if (!planes_ok) return false;
    out.wide.resize(buf.size() / 4);
    memcpy(out.wide.data(), buf.data(), buf.size() * sizeof(uint32_t));
    // Compact triangle records when every leaf holds one triangle: {v1.xyz, rank},
    // {v2.xyz, v3.x}, {v3.yz, 0, 0} (48 B instead of 64 B). The kernel forms e1 = v2 - v1,
    // e2 = v3 - v1 (triangle.h:28, the same float subtractions as above) and the leaf's box
    // as the component min / max of the three vertices, which equals the reference's leaf
    // box (a single triangle's AABB, aabb.h:16-19) as real numbers. A tree whose leaf boxes
    // differ from their triangle's AABB (padded, hand-built or from another builder: the C
    // ABI takes any node array) keeps the 64-B records with the stored box, as does
    // PT_WIDE_COMPACT=0.
    const char* cp = hook_env("PT_WIDE_COMPACT");
    const bool compact = single && tri_boxes && !(cp && *cp == '0');
    if (compact) {
        std::vector<f4> ct(3 * wt_tri.size());
        parallel_chunks(wt_tri.size(), 4096, threads, [&](size_t t0, size_t t1) {
            for (size_t t = t0; t < t1; t++) {
                const float* v = s->verts + 9 * (size_t)s->tri_idx[wt_tri[t]];
                ct[3 * t] = f4{v[0], v[1], v[2], u2f((uint32_t)rank_pos[wt_tri[t]])};
                ct[3 * t + 1] = f4{v[3], v[4], v[5], v[6]};
                ct[3 * t + 2] = f4{v[7], v[8], 0.0f, 0.0f};
            }
        });
        wt = std::move(ct);
    }
    out.wide_compact = compact;
    out.wtris = std::move(wt);
    out.num_wide = (int32_t)queue.size();
    out.wide_width = W;
    out.wide_fmt = fmt;
    for (int a = 0; a < 3; a++) out.wide_span[a] = span[a];
    out.wide_depth = max_level + 1;
    out.wide_single = single;
    // LDS top of tree: the longest prefix of whole levels within the budget
    const char* tb = hook_env("PT_WIDE_TOP_BYTES");
    // default 4 KiB, any index prefix: the root, its children and the first nodes of the
    // third level (BFS order), which most walks read. The launch keeps only as many as fit
    // without costing a block per CU (pt_kernel.hip; config 4: 24 nodes, 3 KiB). Whole
    // levels only (the round-2 rule: 9 nodes) measured 0.7 % slower (profiles/r03y_lds).
    const size_t budget = (tb && *tb) ? (size_t)strtoull(tb, nullptr, 0) : 4096;
    const size_t per = 16 * (size_t)kWideNodeU4(W, fmt);
    int top = 0;
    for (size_t i = 0; i <= queue.size(); i++) {
        if (i == queue.size() || (i > 0 && level[i] != level[i - 1])) {
            if (i * per <= budget) top = (int)i;
            else break;
        }
    }
    // any index prefix that fits (the kernel reads node n from LDS when n < wide_top,
    // whatever its level); PT_WIDE_TOP_PARTIAL=0 (tuning hook): whole levels only
    const char* tp = hook_env("PT_WIDE_TOP_PARTIAL");
    if (!(tp && *tp == '0')) top = (int)std::min(queue.size(), budget / per);
    out.wide_top = top;
    return true;
}

int pack_scene(const pt_scene* s, PackedScene& out) {
    if (!s) return set_error(PT_E_ARG, "scene is NULL");
    if (s->num_tris <= 0) return set_error(PT_E_EMPTY, "No triangles in scene.");
    if (!s->verts || !s->materials || !s->nodes || !s->tri_idx || s->num_nodes <= 0)
        return set_error(PT_E_ARG, "scene arrays must be non-NULL (BVH not built?)");
    const int nn = s->num_nodes, nt = s->num_tris;
    for (int i = 0; i < nt; i++) {
        if (s->tri_idx[i] < 0 || s->tri_idx[i] >= nt)
            return set_error(PT_E_ARG, "tri_idx[%d] = %d out of range", i, s->tri_idx[i]);
    }
    // Walk the tree exactly as BVH::intersect would with every box hit: detects
    // malformed graphs and gives the maximum LIFO occupancy (the kernel's stack).
    std::vector<int32_t> st{0}, depth_of{0};
    std::vector<uint8_t> seen(nn, 0);
    size_t visits = 0;
    int max_sp = 1, max_depth = 0;
    while (!st.empty()) {
        const int n = st.back(), dn = depth_of.back();
        st.pop_back();
        depth_of.pop_back();
        if (seen[n]) return set_error(PT_E_ARG, "BVH node graph is not a tree (node %d reached twice)", n);
        seen[n] = 1;
        visits++;
        max_depth = std::max(max_depth, dn);
        const pt_bvh_node& nd = s->nodes[n];
        if (nd.left == -1 && nd.right == -1) {
            if (nd.tri_start <= nd.tri_end && (nd.tri_start < 0 || nd.tri_end >= nt))
                return set_error(PT_E_ARG, "leaf %d triangle range [%d, %d] out of range", n, nd.tri_start,
                                 nd.tri_end);
            continue;
        }
        if (nd.left < 0 || nd.left >= nn || nd.right < 0 || nd.right >= nn)
            return set_error(PT_E_ARG, "node %d has invalid children (%d, %d)", n, nd.left, nd.right);
        st.push_back(nd.left);
        depth_of.push_back(dn + 1);
        st.push_back(nd.right);
        depth_of.push_back(dn + 1);
        max_sp = std::max(max_sp, (int)st.size());
    }
    out.num_nodes = (int32_t)visits;  // nodes reachable from the root
    out.num_tris = nt;
    out.stack_size = max_sp;
    out.tree_depth = max_depth;
    // Renumber: root -> 0, children of every interior node -> an adjacent pair.
    std::vector<int32_t> newid(nn, -1), order;
    order.reserve(visits);
    newid[0] = 0;
    order.push_back(0);
    for (size_t i = 0; i < order.size(); i++) {
        const pt_bvh_node& nd = s->nodes[order[i]];
        if (nd.left == -1 && nd.right == -1) continue;
        newid[nd.left] = (int32_t)order.size();
        order.push_back(nd.left);
        newid[nd.right] = (int32_t)order.size();
        order.push_back(nd.right);
    }
    // Rank: the order BVH::intersect visits leaves when every box passes (LIFO, left
    // pushed before right, bvh.h:177-178), ascending position inside a leaf. If the
    // leaves partition the positions (always so for BVH::build output), triangles are
    // stored in rank order; otherwise positions are kept and the flat path is off.
    std::vector<int32_t> rank_pos(nt, -1), leaf_nodes;  // old position -> rank position
    bool partition = true;
    {
        int32_t next = 0;
        std::vector<int32_t> st2{0};
        while (!st2.empty()) {
            const int n = st2.back();
            st2.pop_back();
            const pt_bvh_node& nd = s->nodes[n];
            if (nd.left == -1 && nd.right == -1) {
                leaf_nodes.push_back(n);
                for (int i = nd.tri_start; i <= nd.tri_end; i++) {
                    if (rank_pos[i] != -1) partition = false;
                    else rank_pos[i] = next++;
                }
            } else {
                st2.push_back(nd.left);
                st2.push_back(nd.right);
            }
        }
        if (next != nt) partition = false;
        if (!partition)
            for (int i = 0; i < nt; i++) rank_pos[i] = i;
    }
    // Triangle and material records by rank position: independent of the tree work below, so
    // on a thread of their own while it runs (large scenes).
    auto pack_tris = [&] {
        out.coords_small = true;
        for (size_t i = 0; i < 9 * (size_t)nt; i++)
            if (!(fabsf(s->verts[i]) < 0x1p60f)) out.coords_small = false;
        out.tris.resize(3 * (size_t)nt);
        out.mats.resize(2 * (size_t)nt);
        for (int i = 0; i < nt; i++) {
            const int pos = rank_pos[i];
            const int t = s->tri_idx[i];
            const float* v = s->verts + 9 * (size_t)t;
            const v3 v1{v[0], v[1], v[2]}, v2{v[3], v[4], v[5]}, v3_{v[6], v[7], v[8]};
            const v3 e1 = sub(v2, v1), e2 = sub(v3_, v1);
            const v3 n = normalize(cross(e1, e2));
            out.tris[3 * pos] = f4{v1.x, v1.y, v1.z, e1.x};
            out.tris[3 * pos + 1] = f4{e1.y, e1.z, e2.x, e2.y};
            out.tris[3 * pos + 2] = f4{e2.z, n.x, n.y, n.z};
            const pt_material& m = s->materials[t];
            out.mats[2 * pos] = f4{u2f((uint32_t)m.type), m.color[0], m.color[1], m.color[2]};
            out.mats[2 * pos + 1] = f4{m.emit[0], m.emit[1], m.emit[2], m.roughness};
        }
    };
    std::thread tri_worker;
    if (nt >= 4096 && pack_threads() > 1) {
        try {
            tri_worker = std::thread(pack_tris);
        } catch (const std::system_error&) {
        }
    }
    // joined on every return path below (the lambda writes `out`)
    struct JoinOnExit {
        std::thread& t;
        ~JoinOnExit() {
            if (t.joinable()) t.join();
        }
    } join_tris{tri_worker};
    // Containment (child box inside parent box) makes the slab test monotone along
    // every root-leaf chain, which the flat leaf list relies on.
    // (both per node: in chunks on the packing threads)
    std::atomic<bool> contained_all{partition};
    out.nodes.resize(2 * order.size());
    parallel_chunks(order.size(), 16384, order.size() >= 32768 ? pack_threads() : 1, [&](size_t i0, size_t i1) {
        bool ok = true;
        for (size_t i = i0; i < i1; i++) {
            const pt_bvh_node& nd = s->nodes[order[i]];
            const bool leaf = nd.left == -1 && nd.right == -1;
            int32_t a, b;
            if (leaf) {
                a = nd.tri_start <= nd.tri_end ? -(rank_pos[nd.tri_start] + 1) : -1;
                b = nd.tri_start <= nd.tri_end ? rank_pos[nd.tri_end] : -1;
            } else {
                a = newid[nd.left];
                b = 0;
                for (int c : {nd.left, nd.right}) {
                    const pt_bvh_node& ch = s->nodes[c];
                    for (int ax = 0; ax < 3; ax++)
                        if (!(nd.lb[ax] <= ch.lb[ax] && ch.rt[ax] <= nd.rt[ax])) ok = false;
                }
            }
            out.nodes[2 * i] = f4{nd.lb[0], nd.lb[1], nd.lb[2], nd.rt[0]};
            out.nodes[2 * i + 1] = f4{nd.rt[1], nd.rt[2], u2f((uint32_t)a), u2f((uint32_t)b)};
        }
        if (!ok) contained_all = false;
    });
    const bool contained = contained_all;
    out.num_leaves = contained ? (int32_t)leaf_nodes.size() : 0;
    if (contained) {
        out.leaves.resize(2 * leaf_nodes.size());
        for (size_t k = 0; k < leaf_nodes.size(); k++) {
            const pt_bvh_node& nd = s->nodes[leaf_nodes[k]];
            const int32_t first = nd.tri_start <= nd.tri_end ? rank_pos[nd.tri_start] : 0;
            const int32_t last = nd.tri_start <= nd.tri_end ? rank_pos[nd.tri_end] : -1;
            out.leaves[2 * k] = f4{nd.lb[0], nd.lb[1], nd.lb[2], nd.rt[0]};
            out.leaves[2 * k + 1] = f4{nd.rt[1], nd.rt[2], u2f((uint32_t)first), u2f((uint32_t)last)};
        }
    }
    // Wide tree with quantised child boxes, for trees past the flat list's reach.
    // 8-wide by default; PT_WIDE_W=4 selects 4.
    if (contained && !(s->nodes[0].left == -1 && s->nodes[0].right == -1)) {
        const char* we = hook_env("PT_WIDE_W");
        const int W = (we && atoi(we) == 4) ? 4 : 8;
        // binary16 planes by default (one v_fma_mix_f32 per plane instead of a byte
        // conversion and half a packed FMA; config 4 +1.5 %); PT_WIDE_F16=0 keeps bytes
        // PT_WIDE_PLANES=f32 (round 6): the reference's float planes, two children per
        // v_pk_fma_f32; =byte as PT_WIDE_F16=0
        const char* wf = hook_env("PT_WIDE_F16");
        const char* wp = hook_env("PT_WIDE_PLANES");
        int fmt = (wf && *wf == '0') ? kWideByte : kWideF16;
        if (wp && strcmp(wp, "f32") == 0) fmt = kWideF32;
        else if (wp && strcmp(wp, "f16") == 0) fmt = kWideF16;
        else if (wp && strcmp(wp, "byte") == 0) fmt = kWideByte;
        if (!build_wide(s, rank_pos, W, fmt, out)) {
            out.wide.clear();
            out.wtris.clear();
            out.num_wide = 0;
        }
    }
    if (tri_worker.joinable()) tri_worker.join();
    else pack_tris();
    // Wide path: normals with a material id per rank position and the distinct materials
    // (compared bit for bit), so the wide kernel's shading reads one 16-B record per hit
    // and its path records hold material rows of a small table (LDS) instead of triangles.
    if (out.num_wide > 0) {
        out.nrm.resize((size_t)nt);
        std::map<std::array<uint32_t, 8>, int32_t> ids;
        for (int pos = 0; pos < nt; pos++) {
            std::array<uint32_t, 8> key;
            memcpy(key.data(), &out.mats[2 * (size_t)pos], sizeof(key));
            auto it = ids.find(key);
            if (it == ids.end()) {
                it = ids.emplace(key, (int32_t)(out.umats.size() / 2)).first;
                out.umats.push_back(out.mats[2 * (size_t)pos]);
                out.umats.push_back(out.mats[2 * (size_t)pos + 1]);
            }
            const f4& t2 = out.tris[3 * (size_t)pos + 2];
            out.nrm[pos] = f4{t2.y, t2.z, t2.w, u2f((uint32_t)it->second)};
        }
        out.num_umats = (int32_t)(out.umats.size() / 2);
    }
    return PT_OK;
}

}  // namespace pt

using namespace pt;

extern "C" {

int pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_scene_validate(const pt_scene* scene, int32_t info[4]) {
    PackedScene ps;
    const int rc = pack_scene(scene, ps);
    if (rc) return rc;
    if (info) {
        info[0] = ps.num_nodes;
        info[1] = ps.tree_depth;
        info[2] = ps.num_leaves;
        info[3] = ps.stack_size;
    }
    return PT_OK;
}

int pt_scene_info(const pt_scene* scene, int32_t* info, int32_t n) {
    if (!info || n < 0) return set_error(PT_E_ARG, "pt_scene_info: bad argument");
    PackedScene ps;
    const int rc = pack_scene(scene, ps);
    if (rc) return rc;
    const int32_t v[PT_SCENE_INFO_N] = {ps.num_nodes,  ps.tree_depth, ps.num_leaves, ps.stack_size,
                                        ps.num_wide,   ps.wide_width, ps.wide_depth, ps.wide_top,
                                        (int32_t)(ps.wtris.size() / (ps.wide_compact ? 3 : 4)),
                                        ps.num_wide ? (ps.wide_compact ? 48 : 64) : 0};
    for (int32_t i = 0; i < n && i < PT_SCENE_INFO_N; i++) info[i] = v[i];
    return PT_SCENE_INFO_N;
}

// Test hook: FNV-1a (64-bit) of every array and scalar pack_scene produces, so a change to the
// packing's schedule (threads, order of work) can be checked to leave its output bit-identical.
int pt_debug_pack_hash(const pt_scene* scene, uint64_t* hash) {
    if (!hash) return set_error(PT_E_ARG, "pt_debug_pack_hash: hash is NULL");
    PackedScene ps;
    const int rc = pack_scene(scene, ps);
    if (rc) return rc;
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        const unsigned char* c = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
    };
    for (const std::vector<f4>* v : {&ps.nodes, &ps.tris, &ps.mats, &ps.leaves, &ps.wide, &ps.wtris, &ps.nrm, &ps.umats}) {
        const uint64_t n = v->size();
        mix(&n, sizeof(n));
        mix(v->data(), n * sizeof(f4));
    }
    const int32_t sc[] = {ps.num_umats, ps.num_leaves, ps.num_wide, ps.wide_width, ps.wide_depth, ps.wide_top,
                          ps.wide_fmt, ps.wide_single, ps.wide_compact, ps.num_nodes, ps.num_tris, ps.stack_size,
                          ps.tree_depth, ps.coords_small};
    mix(sc, sizeof(sc));
    mix(ps.wide_span, sizeof(ps.wide_span));
    *hash = h;
    return PT_OK;
}

// Test hook: rebuild the wide tree of `scene` and check its format invariants in exact
// arithmetic (__float128: differences of floats within 2^89 of each other are exact):
// every quantised child box contains the reference's box (O + lo 2^e <= lb, O + hi 2^e >=
// rt), inner children are the consecutive nodes from child_base, leaf triangles carry
// their rank and their leaf's exact box, and every triangle is stored exactly once.
// Returns the number of violations (0) or a negative error code.
int pt_debug_wide_verify(const pt_scene* scene, int32_t width) {
    PackedScene ps;
    int rc = pack_scene(scene, ps);
    if (rc) return rc;
    if (width != 4 && width != 8) return set_error(PT_E_ARG, "width must be 4 or 8");
    // rank positions as pack_scene computes them (LIFO walk, left pushed first)
    const int nt = scene->num_tris;
    std::vector<int32_t> rank_pos(nt, -1);
    {
        int32_t next = 0;
        std::vector<int32_t> st{0};
        while (!st.empty()) {
            const int n = st.back();
            st.pop_back();
            const pt_bvh_node& nd = scene->nodes[n];
            if (nd.left == -1 && nd.right == -1) {
                for (int i = nd.tri_start; i <= nd.tri_end; i++) rank_pos[i] = next++;
            } else {
                st.push_back(nd.left);
                st.push_back(nd.right);
            }
        }
    }
    int32_t bad = 0;
    for (const int fmt : {kWideByte, kWideF16, kWideF32}) {  // every plane format
        const bool f16 = fmt == kWideF16, f32 = fmt == kWideF32;
        PackedScene w;
        std::vector<int32_t> slots;
        if (!build_wide(scene, rank_pos, width, fmt, w, &slots)) return set_error(PT_E_ARG, "scene has no wide tree");
        const int U = 4 * kWideNodeU4(width, fmt), QW = width / 4;
        const uint32_t* base = reinterpret_cast<const uint32_t*>(w.wide.data());
        std::vector<int> seen(nt, 0);
        for (int n = 0; n < w.num_wide; n++) {
            const uint32_t* u = base + (size_t)n * U;
            const uint8_t* qb = reinterpret_cast<const uint8_t*>(u + 8);
            const WideHdr hd = wide_hdr(u, fmt);
            const int ni = hd.ni, nl = hd.nl;
            for (int a = 0; a < 3 && fmt == kWideByte; a++)  // the swapped copy of each axis's byte planes matches
                for (int j = 0; j < width; j++) {
                    const uint8_t* b = qb + (size_t)16 * QW * a;
                    if (b[8 * QW + j] != b[4 * QW + j] || b[12 * QW + j] != b[j]) bad++;
                }
            for (int j = ni + nl; j < width && f32; j++)  // empty slots fail every ray: lo = +inf, hi = -inf
                for (int a = 0; a < 3; a++)
                    if (!(u2f(u[4 + 2 * width * a + j]) == INFINITY && u2f(u[4 + 2 * width * a + width + j]) == -INFINITY))
                        bad++;
            for (int j = 0; j < ni + nl; j++) {
                const int b = slots[(size_t)n * width + j];
                if (b < 0) {
                    bad++;
                    continue;
                }
                const pt_bvh_node& nd = scene->nodes[b];
                const bool leaf = nd.left == -1 && nd.right == -1;
                if (leaf != (j >= ni)) bad++;
                for (int a = 0; a < 3; a++) {
                    if (f32) {  // the reference's planes, bit for bit
                        if (u[4 + 2 * width * a + j] != f2u(nd.lb[a]) || u[4 + 2 * width * a + width + j] != f2u(nd.rt[a]))
                            bad++;
                        if (!(fabsf(nd.lb[a]) <= w.wide_span[a] && fabsf(nd.rt[a]) <= w.wide_span[a])) bad++;
                        continue;
                    }
                    const int e = (int)((u[3] >> (8 * a)) & 255u) - 128;
                    const __float128 O = (__float128)u2f(u[a]);
                    const __float128 sc = (__float128)ldexp(1.0, e);
                    const __float128 lo = O + (__float128)wide_plane(u, width, f16, a, j, false) * sc;
                    const __float128 hi = O + (__float128)wide_plane(u, width, f16, a, j, true) * sc;
                    if (!(lo <= (__float128)nd.lb[a]) || !(hi >= (__float128)nd.rt[a])) bad++;
                }
                if (!leaf) continue;
                const uint8_t* ends = hd.ends;
                const int k = j - ni, begin = k ? ends[k - 1] : 0, end = ends[k];
                if (end - begin != nd.tri_end - nd.tri_start + 1) bad++;
                for (int i = nd.tri_start, t = begin; i <= nd.tri_end && t < end; i++, t++) {
                    const float ref[6] = {nd.lb[0], nd.lb[1], nd.lb[2], nd.rt[0], nd.rt[1], nd.rt[2]};
                    const float* v = scene->verts + 9 * (size_t)scene->tri_idx[i];
                    if (w.wide_compact) {
                        // {v1, rank}, {v2, v3.x}, {v3.yz}: the vertices bit for bit, and their
                        // component min / max equal to the reference's leaf box as reals
                        const f4* r = &w.wtris[3 * ((size_t)hd.leaf_base + t)];
                        if (f2u(r[0].w) != (uint32_t)rank_pos[i]) bad++;
                        const float got[9] = {r[0].x, r[0].y, r[0].z, r[1].x, r[1].y, r[1].z, r[1].w, r[2].x, r[2].y};
                        if (memcmp(got, v, sizeof(got)) != 0) bad++;
                        for (int a = 0; a < 3; a++) {
                            if (std::fmin(std::fmin(v[a], v[3 + a]), v[6 + a]) != ref[a]) bad++;
                            if (std::fmax(std::fmax(v[a], v[3 + a]), v[6 + a]) != ref[3 + a]) bad++;
                        }
                    } else {
                        const f4* r = &w.wtris[4 * ((size_t)hd.leaf_base + t)];
                        if (f2u(r[2].y) != (uint32_t)rank_pos[i]) bad++;
                        const float box[6] = {r[2].z, r[2].w, r[3].x, r[3].y, r[3].z, r[3].w};
                        if (memcmp(box, ref, sizeof(box)) != 0) bad++;
                    }
                    seen[i]++;
                }
            }
            // inner slot j is node child_base + j, whose slots are the binary node's subtree
            for (int j = 0; j < ni; j++) {
                const uint32_t c = hd.child_base + (uint32_t)j;
                if (c >= (uint32_t)w.num_wide) {
                    bad++;
                    continue;
                }
                // the child wide node's first slot must descend from binary node slots[n][j]
                const int b = slots[(size_t)n * width + j];
                const pt_bvh_node& nd = scene->nodes[b];
                const int f = slots[(size_t)c * width];
                if (f != nd.left && f != nd.right) {
                    // deeper collapse: f must lie in b's subtree
                    std::vector<int32_t> st{b};
                    bool found = false;
                    while (!st.empty() && !found) {
                        const int x = st.back();
                        st.pop_back();
                        if (x == f) found = true;
                        const pt_bvh_node& xn = scene->nodes[x];
                        if (!(xn.left == -1 && xn.right == -1)) {
                            st.push_back(xn.left);
                            st.push_back(xn.right);
                        }
                    }
                    if (!found) bad++;
                }
            }
        }
        for (int i = 0; i < nt; i++)
            if (seen[i] != 1) bad++;
    }
    return bad;
}

const char* pt_last_error(void) { return g_err.c_str(); }

// One node of the builder's working tree: its idx range, box and children.
struct BuildNode {
    int s0, s1;
    Box box;
    std::unique_ptr<BuildNode> kid[2];
    BuildNode(int a, int b) : s0(a), s1(b) {}
};

// A left subtree of at least kSpawnMin triangles gets a thread of its own while fewer
// than kMaxBuildThreads are building (the reference's SAH often peels a few
// triangles off a large node, so subtree sizes are uneven at any depth).
constexpr int kSpawnMin = 2048;

// BVH::build's loop (bvh.h:79-155) below `t`: box, best split (bvh.h:48-78), the
// reference's two-pointer partition of idx[s0..s1] (bvh.h:124-135, not stable; reproduced
// step by step) and the two children. Node numbers are assigned afterwards.
static void build_subtree(BuildNode* t, std::vector<TriKey>& kord, std::vector<int32_t>& idx) {
    std::vector<BuildNode*> stack{t};
    SplitScratch sc[3];
    std::vector<std::thread> spawned;
    while (!stack.empty()) {
        BuildNode* nd = stack.back();
        stack.pop_back();
        const int s0 = nd->s0, s1 = nd->s1;
        Box box;
        for (int i = s0; i <= s1; i++) box.grow(kord[i].box);
        nd->box = box;
        const Split sp = best_split(kord, s0, s1, sc);
        const int count = s1 - s0 + 1;
        const float nosplit = count * box.half_area();
        if (sp.axis == -1 || sp.cost > nosplit) continue;  // bvh.h:104-109
        int a = s0, b = s1, lcount = 0;
        while (a < b) {
            if (kord[a].c[sp.axis] < sp.value) {
                a++;
                lcount++;
            } else if (kord[b].c[sp.axis] >= sp.value) {
                b--;
            } else {
                std::swap(idx[a], idx[b]);
                std::swap(kord[a], kord[b]);
            }
        }
        if (lcount == 0 || lcount == count) continue;
        nd->kid[0].reset(new BuildNode(s0, s0 + lcount - 1));
        nd->kid[1].reset(new BuildNode(s0 + lcount, s1));
        for (auto& k : nd->kid) {
            bool own = false;
            if (&k == &nd->kid[0] && k->s1 - k->s0 + 1 >= kSpawnMin) {
                if (g_build_threads.fetch_add(1) < kMaxBuildThreads) {
                    try {
                        spawned.emplace_back([&kord, &idx](BuildNode* b) {
                            build_subtree(b, kord, idx);
                            g_build_threads.fetch_sub(1);
                        }, k.get());
                        own = true;
                    } catch (const std::system_error&) {  // no thread: built on this one
                    }
                }
                if (!own) g_build_threads.fetch_sub(1);
            }
            if (!own) stack.push_back(k.get());
        }
    }
    for (auto& th : spawned) th.join();
}

// build_subtree over the sorted per-axis lists (the default): the reference's partition on
// positions (bvh.h:124-135, reproduced step by step, `where` kept up to date), then every
// axis's segment split stably by the new positions: left child = positions [s0, s0 + lcount).
static void build_subtree_sorted(BuildNode* t, SortedBuild& B) {
    std::vector<BuildNode*> stack{t};
    SortedScratch sc[3];
    std::vector<std::thread> spawned;
    std::vector<int32_t>& idx = B.idx;
    const TriKey* key = B.key.data();
    while (!stack.empty()) {
        BuildNode* nd = stack.back();
        stack.pop_back();
        const int s0 = nd->s0, s1 = nd->s1;
        Box box;
        for (int i = s0; i <= s1; i++) box.grow(key[idx[i]].box);  // position order, as the reference
        nd->box = box;
        const Split sp = sorted_best_split(B, s0, s1, sc);
        const int count = s1 - s0 + 1;
        const float nosplit = count * box.half_area();
        if (sp.axis == -1 || sp.cost > nosplit) continue;  // bvh.h:104-109
        int a = s0, b = s1, lcount = 0;
        while (a < b) {
            if (key[idx[a]].c[sp.axis] < sp.value) {
                a++;
                lcount++;
            } else if (key[idx[b]].c[sp.axis] >= sp.value) {
                b--;
            } else {
                std::swap(idx[a], idx[b]);
                B.where[idx[a]] = a;
                B.where[idx[b]] = b;
            }
        }
        if (lcount == 0 || lcount == count) continue;
        const int mid = s0 + lcount;
        std::vector<int32_t>& tmp = sc[0].tmp;
        tmp.resize(count);
        for (int ax = 0; ax < 3; ax++) {  // stable split of the axis's segment by position
            int32_t* seg = B.sorted[ax].data() + s0;
            int l = 0, r = lcount;
            for (int k = 0; k < count; k++) {
                const int32_t e = seg[k];
                tmp[B.where[e] < mid ? l++ : r++] = e;
            }
            memcpy(seg, tmp.data(), sizeof(int32_t) * (size_t)count);
        }
        nd->kid[0].reset(new BuildNode(s0, mid - 1));
        nd->kid[1].reset(new BuildNode(mid, s1));
        for (auto& k : nd->kid) {
            bool own = false;
            if (&k == &nd->kid[0] && k->s1 - k->s0 + 1 >= kSpawnMin) {
                if (g_build_threads.fetch_add(1) < kMaxBuildThreads) {
                    try {
                        spawned.emplace_back([&B](BuildNode* c) {
                            build_subtree_sorted(c, B);
                            g_build_threads.fetch_sub(1);
                        }, k.get());
                        own = true;
                    } catch (const std::system_error&) {  // no thread: built on this one
                    }
                }
                if (!own) g_build_threads.fetch_sub(1);
            }
            if (!own) stack.push_back(k.get());
        }
    }
    for (auto& th : spawned) th.join();
}

// Iterative teardown (a degenerate tree is as deep as it has triangles).// Iterative teardown (a degenerate tree is as deep as it has triangles).
static void free_subtree(BuildNode& root) {
    std::vector<std::unique_ptr<BuildNode>> pending;
    for (auto& k : root.kid) if (k) pending.push_back(std::move(k));
    while (!pending.empty()) {
        std::unique_ptr<BuildNode> b = std::move(pending.back());
        pending.pop_back();
        for (auto& k : b->kid) if (k) pending.push_back(std::move(k));
    }
}

int pt_bvh_build(int32_t n, const float* verts, pt_bvh_node* nodes_out, int32_t* idx_out) {
    if (n <= 0) return set_error(PT_E_EMPTY, "No triangles in scene.");
    if (!verts || !nodes_out || !idx_out) return set_error(PT_E_ARG, "pt_bvh_build: NULL argument");
    for (size_t i = 0; i < 9 * (size_t)n; i++)
        if (!isfinite(verts[i])) return set_error(PT_E_ARG, "pt_bvh_build: non-finite vertex coordinate");
    std::vector<TriKey> keys(n);
    for (int i = 0; i < n; i++) {
        const float* v = verts + 9 * (size_t)i;
        const v3 a{v[0], v[1], v[2]}, b{v[3], v[4], v[5]}, c{v[6], v[7], v[8]};
        const v3 ctr = add(add(a, b), c);
        keys[i].c[0] = ctr.x / 3.0f;
        keys[i].c[1] = ctr.y / 3.0f;
        keys[i].c[2] = ctr.z / 3.0f;
        keys[i].box.grow(a);
        keys[i].box.grow(b);
        keys[i].box.grow(c);
    }
    std::vector<int32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    // Subtrees are independent (each owns its idx range), so they are built in parallel;
    // the reference numbers nodes in the order its LIFO loop splits them (bvh.h:137-152),
    // which the replay below reproduces from the finished topology.
    BuildNode root(0, n - 1);
    // PT_BUILD_RESORT=1 (tuning hook): the round-5 builder, which sorts every node's axes again
    const char* rs = hook_env("PT_BUILD_RESORT");
    if (rs && *rs == '1') {
        build_subtree(&root, keys, idx);  // keys start in idx order (identity) and move with it
    } else {
        SortedBuild B(keys, idx);
        B.where.resize(n);
        std::iota(B.where.begin(), B.where.end(), 0);
        {
            Helper h1([&] { sort_axis(B, 1); }), h2([&] { sort_axis(B, 2); });
            sort_axis(B, 0);
            if (!h1.running()) sort_axis(B, 1);
            if (!h2.running()) sort_axis(B, 2);
        }
        build_subtree_sorted(&root, B);
    }
    std::vector<pt_bvh_node> nodes;
    nodes.reserve(2 * (size_t)n);
    auto emit = [&](const BuildNode* b) {
        pt_bvh_node nd;
        memset(&nd, 0, sizeof(nd));
        nd.lb[0] = b->box.lb.x; nd.lb[1] = b->box.lb.y; nd.lb[2] = b->box.lb.z;
        nd.rt[0] = b->box.rt.x; nd.rt[1] = b->box.rt.y; nd.rt[2] = b->box.rt.z;
        nd.left = nd.right = -1;
        nd.tri_start = b->s0;
        nd.tri_end = b->s1;
        nodes.push_back(nd);
        return (int)nodes.size() - 1;
    };
    emit(&root);
    std::vector<std::pair<const BuildNode*, int>> replay{{&root, 0}};
    while (!replay.empty()) {
        const BuildNode* b = replay.back().first;
        const int ci = replay.back().second;
        replay.pop_back();
        if (!b->kid[0]) continue;
        const int L = emit(b->kid[0].get());
        const int R = emit(b->kid[1].get());
        nodes[ci].left = L;
        nodes[ci].right = R;
        replay.push_back({b->kid[0].get(), L});
        replay.push_back({b->kid[1].get(), R});
    }
    free_subtree(root);
    memcpy(nodes_out, nodes.data(), nodes.size() * sizeof(pt_bvh_node));
    memcpy(idx_out, idx.data(), idx.size() * sizeof(int32_t));
    return (int)nodes.size();
}

int pt_camera_init(const float pos[3], const float forward[3], const float up[3], int32_t res_x,
                   int32_t res_y, float fov, float distance, pt_camera* out) {
    if (!pos || !forward || !up || !out) return set_error(PT_E_ARG, "pt_camera_init: NULL argument");
    if (res_x <= 0 || res_y <= 0) return set_error(PT_E_ARG, "pt_camera_init: resolution must be positive");
    const v3 f0{forward[0], forward[1], forward[2]}, u0{up[0], up[1], up[2]};
    const v3 fw = normalize(f0);
    const v3 right = normalize(cross(f0, u0));  // camera.h:37 uses the un-normalised arguments
    const v3 upn = normalize(u0);
    if (fabsf(dot(fw, upn)) > 0.999)
        return set_error(PT_E_ARG, "Up vector is too close to forward vector");
    memset(out, 0, sizeof(*out));
    out->pos[0] = pos[0];
    out->pos[1] = pos[1];
    out->pos[2] = pos[2];
    out->res[0] = res_x;
    out->res[1] = res_y;
    const float half_tan = tanf(fov / 2);
    out->v_res[0] = 2 * distance * half_tan;
    out->v_res[1] = 2 * distance * half_tan * res_y / res_x;
    out->cell_size = out->v_res[0] / res_x;
    out->distance = distance;
    const float rows[9] = {right.x, right.y, right.z, upn.x, upn.y, upn.z, -fw.x, -fw.y, -fw.z};
    memcpy(out->transform, rows, sizeof(rows));
    return PT_OK;
}

int32_t pt_part_rows(int32_t res_y, int32_t part_index, int32_t part_count, int32_t band_rows) {
    if (res_y <= 0 || part_count <= 0 || band_rows <= 0 || part_index < 0 || part_index >= part_count) return 0;
    int32_t rows = 0;
    for (int32_t band = part_index; band * band_rows < res_y; band += part_count)
        rows += std::min(band_rows, res_y - band * band_rows);
    return rows;
}

// One value of gamma_correct + save_png (image.h:41-55; clamp = std::max(min, std::min(max,
// x)), linalg.h:233-235): powf, clamp to [0, 1], * 255, truncate.
static inline uint8_t quant8(float x, float inv) {
    float y = powf(x, inv);
    y = (y < 1.0f) ? y : 1.0f;  // std::min(max, x)
    y = (0.0f < y) ? y : 0.0f;  // std::max(min, .)
    return (uint8_t)(y * 255);
}

int pt_rgb8_thresholds(float gamma, float* thr, int32_t* neg_mode) {
    if (!thr) return set_error(PT_E_ARG, "pt_rgb8_thresholds: thr is NULL");
    const float inv = 1 / gamma;  // image.h:43
    if (!(inv > 0.0f) || !(inv < __builtin_inff()))
        return set_error(PT_E_ARG, "pt_rgb8_thresholds: gamma must be positive and finite");
    for (int k = 1; k <= 255; k++) {
        uint32_t lo = 0, hi = 0x7f800000u;  // quant8(+0) = 0 < k <= quant8(+inf) = 255
        while (hi - lo > 1) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (quant8(u2f(mid), inv) >= k) hi = mid;
            else lo = mid;
        }
        thr[k - 1] = u2f(hi);
    }
    if (neg_mode) *neg_mode = (floorf(inv) != inv) ? 0 : (fmodf(inv, 2.0f) == 1.0f ? 1 : 2);
    return PT_OK;
}

int pt_image_to_rgb8(const float* lin, int32_t w, int32_t h, float gamma, uint8_t* rgb8) {
    if (!lin || !rgb8 || w <= 0 || h <= 0) return set_error(PT_E_ARG, "pt_image_to_rgb8: bad argument");
    const float inv = 1 / gamma;  // image.h:43 pow(pixel, 1 / gamma)
    for (int32_t row = 0; row < h; row++) {
        const float* src = lin + (size_t)(h - row - 1) * w * 3;  // vertical flip, image.h:51
        uint8_t* dst = rgb8 + (size_t)row * w * 3;
        for (int32_t i = 0; i < 3 * w; i++) {
            dst[i] = quant8(src[i], inv);
        }
    }
    return PT_OK;
}

static void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

static void put_chunk(std::vector<uint8_t>& f, const char* type, const uint8_t* data, size_t n) {
    put_be32(f, (uint32_t)n);
    size_t at = f.size();
    f.insert(f.end(), type, type + 4);
    if (n) f.insert(f.end(), data, data + n);
    uLong crc = crc32(0L, f.data() + at, (uInt)(n + 4));
    put_be32(f, (uint32_t)crc);
}

int pt_write_png(const char* filename, const uint8_t* rgb8, int32_t w, int32_t h) {
    if (!filename || !rgb8 || w <= 0 || h <= 0) return set_error(PT_E_ARG, "pt_write_png: bad argument");
    std::vector<uint8_t> raw((size_t)h * (3 * (size_t)w + 1));
    for (int32_t r = 0; r < h; r++) {
        raw[(size_t)r * (3 * w + 1)] = 0;  // filter: none
        memcpy(&raw[(size_t)r * (3 * w + 1) + 1], rgb8 + (size_t)r * 3 * w, 3 * (size_t)w);
    }
    uLongf zlen = compressBound(raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), raw.size(), 6) != Z_OK)
        return set_error(PT_E_IO, "Failed to write image to file: %s", filename);
    std::vector<uint8_t> f = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    uint8_t ihdr[13];
    ihdr[0] = (uint8_t)(w >> 24); ihdr[1] = (uint8_t)(w >> 16); ihdr[2] = (uint8_t)(w >> 8); ihdr[3] = (uint8_t)w;
    ihdr[4] = (uint8_t)(h >> 24); ihdr[5] = (uint8_t)(h >> 16); ihdr[6] = (uint8_t)(h >> 8); ihdr[7] = (uint8_t)h;
    ihdr[8] = 8;   // bit depth
    ihdr[9] = 2;   // colour type RGB
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    put_chunk(f, "IHDR", ihdr, 13);
    put_chunk(f, "IDAT", z.data(), zlen);
    put_chunk(f, "IEND", nullptr, 0);
    FILE* fp = fopen(filename, "wb");
    if (!fp) return set_error(PT_E_IO, "Failed to write image to file: %s", filename);
    size_t wr = fwrite(f.data(), 1, f.size(), fp);
    int rc = fclose(fp);
    if (wr != f.size() || rc != 0) return set_error(PT_E_IO, "Failed to write image to file: %s", filename);
    return PT_OK;
}

}  // extern "C"
