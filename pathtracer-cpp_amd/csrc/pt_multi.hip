// pt_multi.hip — one process, several GPUs: the frame's row bands rendered on every
// listed device and gathered to the first one. Replaces the
// reference's GL tile loop (render.h:128-139: tiles drawn one by one on one context).
//
//   parts     row h belongs to part (h / band) % n (pt_part_rows); part p renders on
//             devices[p] from its own host thread and context, into a device buffer
//   gather    distinct devices: one RCCL group of point-to-point sends, part p's
//             buffer -> device 0 (ncclCommInitAll over the device list, cached for the
//             process; librccl is dlopen'ed on first use, so single-GPU users never load
//             it), then pt_assemble_kernel puts every row in place on device 0 and one
//             D2H copy returns the frame (or its 8-bit PNG bytes: pt_render_rgb8_devices)
//             a device listed twice (RCCL rejects duplicate GPUs in one communicator) or
//             no RCCL: each part is copied to the host and the rows are placed there
// Per-sample seeding makes every pixel independent of the partition, so the image is
// bit-identical for any device list.
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <dlfcn.h>
#include <signal.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pt_hip_debug.h"
#include "pt_internal.h"

namespace pt {

// Diagnostics (PT_SEGV_TRACE=1, read at library load): a SIGSEGV prints the faulting thread's
// native backtrace (symbol names where the libraries export them) to stderr before the
// default action, to place a crash seen only at process exit.
// A fault at a PC outside any code (a call through a destroyed object) cannot be unwound by
// backtrace(); the handler then also prints the interrupted thread's PC and the stack words
// that point into a loaded library (return addresses), resolved by dladdr.
namespace {
void segv_put(const char* s) { (void)!write(2, s, strlen(s)); }
void segv_addr(const void* a) {
    char buf[512];
    Dl_info di;
    if (dladdr(a, &di) && di.dli_fname) {
        const unsigned long off = (unsigned long)((const char*)a - (const char*)di.dli_fbase);
        snprintf(buf, sizeof(buf), "  %p %s+0x%lx %s\n", a, di.dli_fname, off, di.dli_sname ? di.dli_sname : "");
    } else {
        snprintf(buf, sizeof(buf), "  %p (no library)\n", a);
    }
    segv_put(buf);
}
void segv_trace(int sig, siginfo_t* si, void* uc_) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    char buf[160];
    snprintf(buf, sizeof(buf), "[pt] SIGSEGV at %p in thread %ld, native backtrace:\n", si ? si->si_addr : nullptr,
             (long)syscall(SYS_gettid));
    segv_put(buf);
    backtrace_symbols_fd(frames, n, 2);
    const ucontext_t* uc = static_cast<const ucontext_t*>(uc_);
    const void* pc = (const void*)uc->uc_mcontext.gregs[REG_RIP];
    const uintptr_t* sp = (const uintptr_t*)uc->uc_mcontext.gregs[REG_RSP];
    segv_put("[pt] interrupted PC:\n");
    segv_addr(pc);
    segv_put("[pt] code addresses on the interrupted stack:\n");
    for (int i = 0, shown = 0; i < 512 && shown < 24; i++) {
        Dl_info di;
        if (dladdr((const void*)sp[i], &di) && di.dli_fname) {
            segv_addr((const void*)sp[i]);
            shown++;
        }
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
void segv_install() {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
}
struct SegvTraceInstaller {
    SegvTraceInstaller() {
        const char* e = getenv("PT_SEGV_TRACE");
        if (e && *e == '1') segv_install();
    }
} g_segv_trace_installer;
}  // namespace

// frame row h <- row (h / (band * parts)) * band + h % band of part (h / band) % parts,
// parts stacked [parts][max_rows][W * 3] in `gathered`
__global__ __launch_bounds__(256) void pt_assemble_kernel(const float* __restrict__ gathered,
                                                          float* __restrict__ frame, int W, int parts, int band,
                                                          int max_rows) {
    const int h = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= 3 * W) return;
    const int kb = h / band;
    const int p = kb % parts, i = (kb / parts) * band + h % band;
    frame[(size_t)h * 3 * W + c] = gathered[((size_t)p * max_rows + i) * 3 * W + c];
}

namespace {

// RCCL entry points, resolved from librccl.so.1 on first use.
struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    // teardown of a failed set (either may be missing from an old librccl; abort first)
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
};

Rccl& rccl() {
    static Rccl* r = [] {
        Rccl* x = new Rccl();
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            x->why = std::string("librccl not loadable: ") + dlerror();
            return x;
        }
        x->comm_init_all = (decltype(x->comm_init_all))dlsym(h, "ncclCommInitAll");
        x->group_start = (decltype(x->group_start))dlsym(h, "ncclGroupStart");
        x->group_end = (decltype(x->group_end))dlsym(h, "ncclGroupEnd");
        x->send = (decltype(x->send))dlsym(h, "ncclSend");
        x->recv = (decltype(x->recv))dlsym(h, "ncclRecv");
        x->error_string = (decltype(x->error_string))dlsym(h, "ncclGetErrorString");
        x->comm_abort = (decltype(x->comm_abort))dlsym(h, "ncclCommAbort");
        x->comm_destroy = (decltype(x->comm_destroy))dlsym(h, "ncclCommDestroy");
        x->ok = x->comm_init_all && x->group_start && x->group_end && x->send && x->recv && x->error_string &&
                (x->comm_abort || x->comm_destroy);
        if (!x->ok) x->why = "librccl lacks a needed symbol";
        return x;
    }();
    return *r;
}

// The table in use: librccl's, or a test's fakes (pt_debug_rccl_failover) while it runs.
Rccl* g_rccl_fake = nullptr;
Rccl& rccl_table() { return g_rccl_fake ? *g_rccl_fake : rccl(); }

// One communicator per device of a device list, created once per process (init costs
// hundreds of ms) and kept: RCCL communicators are not torn down at exit. Each set has
// its own mutex, held from ncclGroupStart until the gather's stream is drained: two host
// threads rendering over the same device list must not interleave groups on the same
// communicators. A set whose group failed is dropped from the cache and every one of its
// communicators aborted (ncclCommAbort; ncclCommDestroy where abort is missing), so no
// live communicator with operations in flight is left behind; the next call makes a fresh
// set, and the failing call assembles the frame on the host (pt_stats.gather_path =
// PT_GATHER_HOST_FALLBACK, one stderr line per such frame).
struct CommSet {
    std::vector<ncclComm_t> comms;
    std::mutex mu;
    bool failed = false;  // aborted (fail_comms): a thread that took mu after that must not use comms
};
std::mutex g_comm_mu;
std::map<std::vector<int32_t>, std::shared_ptr<CommSet>> g_comms;

// Abort (or destroy) every communicator of a set; returns how many were torn down.
int abort_comms(Rccl& R, std::vector<ncclComm_t>& comms) {
    int n = 0;
    for (ncclComm_t& c : comms) {
        if (!c) continue;
        if (R.comm_abort) (void)R.comm_abort(c);
        else if (R.comm_destroy) (void)R.comm_destroy(c);
        c = nullptr;
        n++;
    }
    return n;
}

int get_comms(const std::vector<int32_t>& devs, std::shared_ptr<CommSet>& out) {
    Rccl& R = rccl_table();
    if (!R.ok) return set_error(PT_E_HIP, "%s", R.why.c_str());
    std::lock_guard<std::mutex> lock(g_comm_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        auto cs = std::make_shared<CommSet>();
        cs->comms.assign(devs.size(), nullptr);
        // RCCL prints its version banner to stdout at init; the drop-in's stdout is the
        // reference's console contract (render.h:79-101), so the banner goes to stderr.
        // The redirect is process-wide for the duration of ncclCommInitAll: no other host
        // thread may write to stdout during the first multi-device render of a device list
        // (the drop-in's render_cpu / render_gpu print only from the calling thread, before
        // and after it).
        fflush(stdout);
        const int saved = dup(1);
        if (saved >= 0) dup2(2, 1);
        const ncclResult_t r = R.comm_init_all(cs->comms.data(), (int)devs.size(), devs.data());
        fflush(stdout);
        if (saved >= 0) {
            dup2(saved, 1);
            close(saved);
        }
        if (r != ncclSuccess) {
            abort_comms(R, cs->comms);  // whatever a failed init left behind
            return set_error(PT_E_HIP, "ncclCommInitAll: %s", R.error_string(r));
        }
        it = g_comms.emplace(devs, std::move(cs)).first;
    }
    out = it->second;
    return PT_OK;
}

// A set whose group failed: out of the cache, every communicator aborted. The caller holds
// cs->mu (no other thread can be inside a group on these communicators). Returns the number
// of communicators torn down.
int fail_comms(const std::vector<int32_t>& devs, const std::shared_ptr<CommSet>& cs) {
    cs->failed = true;  // under cs->mu: threads waiting on it see the flag when they get it
    {
        std::lock_guard<std::mutex> lock(g_comm_mu);
        auto it = g_comms.find(devs);
        if (it != g_comms.end() && it->second == cs) g_comms.erase(it);
    }
    return abort_comms(rccl_table(), cs->comms);
}

// One RCCL group: part p's buffer (send[p] on stream sstream[p]) -> recv[p] on device 0's
// stream (p = 0 is RCCL's send-to-self). The group is ended even after a failed call, as
// RCCL requires.
ncclResult_t group_gather(Rccl& R, CommSet& cs, int n, const std::vector<const void*>& send,
                          const std::vector<void*>& recv, size_t count, const std::vector<hipStream_t>& sstream,
                          hipStream_t rstream) {
    ncclResult_t r = R.group_start();
    if (r != ncclSuccess) return r;
    for (int p = 0; p < n && r == ncclSuccess; p++) r = R.send(send[p], count, ncclFloat32, 0, cs.comms[p], sstream[p]);
    for (int p = 0; p < n && r == ncclSuccess; p++) r = R.recv(recv[p], count, ncclFloat32, p, cs.comms[0], rstream);
    const ncclResult_t re = R.group_end();
    return r == ncclSuccess ? re : r;
}

// Why a gather over distinct devices went through the host: one stderr line per frame so
// assembled (the frame is still bit-identical; pt_stats.gather_path says which way it went).
void note_host_gather(const std::string& why) {
    fprintf(stderr, "[libpt_hip] RCCL gather unavailable (%s); parts assembled on the host\n", why.c_str());
}

#define HIP_OK(expr)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) return set_error(PT_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// The parts' progress reports (pt_params.progress) summed into one stream for the
// caller: reports arrive from the parts' threads, the caller's callback sees them one at
// a time with the done count of all parts.
struct Progress {
    std::mutex mu;
    pt_progress_fn fn = nullptr;
    void* user = nullptr;
    int64_t total = 0, reported = 0;
    std::vector<int64_t> done;
};
struct PartProgress {
    Progress* agg;
    int part;
};

void part_progress(void* u, int64_t done, int64_t) {
    PartProgress* pp = static_cast<PartProgress*>(u);
    Progress& g = *pp->agg;
    std::lock_guard<std::mutex> lock(g.mu);
    g.done[pp->part] = done;
    int64_t sum = 0;
    for (int64_t d : g.done) sum += d;
    if (sum > g.reported) {
        g.reported = sum;
        g.fn(g.user, sum, g.total);
    }
}

// A part's context and its device output buffer (max_rows * W * 3 floats: every part's
// buffer has the gather's common size), kept between calls in a DevSet.
struct Part {
    pt_ctx* ctx = nullptr;
    float* d_out = nullptr;
    size_t out_cap = 0;  // floats d_out holds
    pt_stats st{};
    int rc = PT_OK;
    std::string err;
    double render_ms = 0.0;
};

// The contexts of one device list, kept for the process (pt_devices_release frees them):
// a render on the same list reuses them (no context creation) and uploads the scene again
// only when its arrays differ from the ones the contexts hold (`scene` is an exact copy of
// them, compared byte for byte). `mu` is held for a whole render; a second host thread
// rendering on the same list meanwhile gets fresh contexts of its own for that call.
// The gather's buffers on the first device (d_gather: every part's rows, d_frame: the
// assembled frame, d_rgb8: its bytes) are kept too, grown as needed: config 5 allocated
// 2 x 201 MB per frame before. The contexts' radiance slabs, the large buffers,
// are released after every render (ctx_release_slabs; ADVICE r5: a caller that renders once
// and then allocates must get that memory back without pt_devices_release).
struct DevSet {
    std::mutex mu;
    std::vector<Part> parts;
    std::vector<uint8_t> scene;  // the scene the contexts hold ("" = none or unknown)
    int dev0 = -1;               // the device the gather buffers live on
    float* d_gather = nullptr;
    size_t gather_cap = 0;       // floats
    float* d_frame = nullptr;
    size_t frame_cap = 0;        // floats
    uint8_t* d_rgb8 = nullptr;
    size_t rgb8_cap = 0;         // bytes
};

// A buffer of at least `n` elements on the current device, kept in (*p, *cap).
template <typename T>
int grow(T** p, size_t* cap, size_t n) {
    if (*p && *cap >= n) return PT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        return set_error(PT_E_HIP, "hipMalloc of %zu gather bytes failed", n * sizeof(T));
    }
    *cap = n;
    return PT_OK;
}

void free_gather(DevSet& set) {
    if (set.dev0 >= 0) (void)hipSetDevice(set.dev0);
    for (void* p : {(void*)set.d_gather, (void*)set.d_frame, (void*)set.d_rgb8})
        if (p) (void)hipFree(p);
    set.d_gather = set.d_frame = nullptr;
    set.d_rgb8 = nullptr;
    set.gather_cap = set.frame_cap = set.rgb8_cap = 0;
    set.dev0 = -1;
}
std::mutex g_dev_sets_mu;
std::map<std::vector<int32_t>, std::shared_ptr<DevSet>> g_dev_sets;
std::atomic<int64_t> g_upload_skips{0};

// The bytes that define a scene for the device: counts and every array pt_ctx_set_scene reads.
std::vector<uint8_t> scene_bytes(const pt_scene* s) {
    std::vector<uint8_t> b;
    if (!s || s->num_tris <= 0 || s->num_nodes <= 0 || !s->verts || !s->materials || !s->nodes || !s->tri_idx) return b;
    auto put = [&b](const void* p, size_t n) {
        const uint8_t* q = static_cast<const uint8_t*>(p);
        b.insert(b.end(), q, q + n);
    };
    put(&s->num_tris, sizeof(s->num_tris));
    put(&s->num_nodes, sizeof(s->num_nodes));
    put(s->verts, sizeof(float) * 9 * (size_t)s->num_tris);
    put(s->materials, sizeof(pt_material) * (size_t)s->num_tris);
    put(s->nodes, sizeof(pt_bvh_node) * (size_t)s->num_nodes);
    put(s->tri_idx, sizeof(int32_t) * (size_t)s->num_tris);
    // under PT_TEST_HOOKS=1 the packing depends on tuning hooks too (PT_WIDE_W, ...):
    // every PT_* variable is part of the key, so a test that changes one uploads again
    if (hook_env("PT_TEST_HOOKS"))
        for (char** e = environ; *e; e++)
            if (strncmp(*e, "PT_", 3) == 0) put(*e, strlen(*e) + 1);
    return b;
}

void free_part(Part& P, int device) {
    if (P.d_out) {
        (void)hipSetDevice(device);
        (void)hipFree(P.d_out);
    }
    if (P.ctx) pt_ctx_destroy(P.ctx);
    P = Part();
}

// Render part p of the partition on devices[p] into parts[p].d_out (device memory), creating
// the part's context and buffer if it has none and uploading the scene if `upload`.
void render_part(const pt_scene* scene, const pt_camera* cam, const pt_params* params, const int32_t* devices,
                 int n, int band, size_t part_floats, bool upload, Part& P, int p, PartProgress* pp) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc = P.ctx ? PT_OK : pt_ctx_create(devices[p], &P.ctx);
    if (!rc && upload) rc = pt_ctx_set_scene(P.ctx, scene);
    if (!rc && hipSetDevice(devices[p]) != hipSuccess) rc = set_error(PT_E_HIP, "hipSetDevice failed");
    if (!rc && P.out_cap < part_floats) {
        if (P.d_out) (void)hipFree(P.d_out);
        P.d_out = nullptr;
        P.out_cap = 0;
        if (hipMalloc((void**)&P.d_out, std::max<size_t>(part_floats, 1) * sizeof(float)) != hipSuccess)
            rc = set_error(PT_E_HIP, "hipMalloc of the part buffer failed");
        else
            P.out_cap = part_floats;
    }
    if (!rc) {
        pt_params q = *params;
        q.part_index = p;
        q.part_count = n;
        q.band_rows = band;
        q.progress = params->progress ? part_progress : nullptr;
        q.progress_user = pp;
        memset(&P.st, 0, sizeof(P.st));
        if (pt_part_rows(cam->res[1], p, n, band) > 0) rc = pt_ctx_render(P.ctx, cam, &q, P.d_out, 1, &P.st);
    }
    P.render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc) P.err = pt_last_error();
    P.rc = rc;
}

void release(std::vector<Part>& parts, const int32_t* devices) {
    for (size_t p = 0; p < parts.size(); p++) free_part(parts[p], devices[p]);
}

// The cached set of a device list, locked for this call; or, when another thread is
// rendering on it, a fresh set of this call's own (`cached` false: freed at the end).
std::shared_ptr<DevSet> take_set(const std::vector<int32_t>& devs, std::unique_lock<std::mutex>& lock, bool& cached) {
    std::shared_ptr<DevSet> set;
    const char* ce = hook_env("PT_DEVICES_CACHE");  // test hook: 0 = fresh contexts every call (A/B)
    if (ce && *ce == '0') {
        cached = false;
        set = std::make_shared<DevSet>();
        lock = std::unique_lock<std::mutex>(set->mu);
        set->parts.assign(devs.size(), Part());
        return set;
    }
    {
        std::lock_guard<std::mutex> g(g_dev_sets_mu);
        auto it = g_dev_sets.find(devs);
        if (it == g_dev_sets.end()) it = g_dev_sets.emplace(devs, std::make_shared<DevSet>()).first;
        set = it->second;
    }
    lock = std::unique_lock<std::mutex>(set->mu, std::try_to_lock);
    cached = lock.owns_lock();
    if (!cached) {
        set = std::make_shared<DevSet>();
        lock = std::unique_lock<std::mutex>(set->mu);
    }
    if (set->parts.size() != devs.size()) {
        free_gather(*set);
        release(set->parts, devs.data());
        set->parts.assign(devs.size(), Part());
        set->scene.clear();
    }
    set->dev0 = devs[0];
    return set;
}

// A failed render leaves no half-updated contexts behind: the set is emptied and dropped.
void drop_set(const std::vector<int32_t>& devs, DevSet& set) {
    free_gather(set);
    release(set.parts, devs.data());
    set.parts.clear();
    set.scene.clear();
}

// out_rgb (H*W*3 floats, h = 0 first) and/or out_rgb8 (H*W*3 bytes, top row first,
// gamma + quantisation as pt_image_to_rgb8) may be NULL.
int render_devices(const pt_scene* scene, const pt_camera* cam, const pt_params* params, const int32_t* devices,
                   int32_t n_devices, float* out_rgb, uint8_t* out_rgb8, float gamma, pt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!params || !cam || !devices || n_devices <= 0 || (!out_rgb && !out_rgb8))
        return set_error(PT_E_ARG, "pt_render_*_devices: bad argument");
    if (n_devices > PT_MAX_DEVICES) return set_error(PT_E_ARG, "at most %d devices", PT_MAX_DEVICES);
    if (scene && scene->num_tris <= 0) return set_error(PT_E_EMPTY, "No triangles in scene.");
    const int W = cam->res[0], H = cam->res[1];
    if (W <= 0 || H <= 0) return set_error(PT_E_ARG, "camera resolution must be positive");
    if (H > 65535) return set_error(PT_E_ARG, "%d rows exceed the assembly grid", H);
    const int n = n_devices, band = params->band_rows > 0 ? params->band_rows : 1;
    int max_rows = 0;
    for (int p = 0; p < n; p++) max_rows = std::max(max_rows, (int)pt_part_rows(H, p, n, band));
    const size_t part_floats = (size_t)max_rows * W * 3;
    std::vector<int32_t> devs(devices, devices + n);
    std::unique_lock<std::mutex> set_lock;
    bool cached = false;
    std::shared_ptr<DevSet> set = take_set(devs, set_lock, cached);
    std::vector<Part>& parts = set->parts;
    std::vector<uint8_t> key = scene_bytes(scene);
    const bool upload = key.empty() || key != set->scene;
    if (!upload) g_upload_skips += n;
    set->scene.clear();  // until every part holds the new scene
    Progress prog;
    prog.fn = params->progress;
    prog.user = params->progress_user;
    prog.total = (int64_t)W * H * std::max(params->spp, 0);
    prog.done.assign(n, 0);
    std::vector<PartProgress> pp(n);
    for (int p = 0; p < n; p++) pp[p] = PartProgress{&prog, p};
    {
        std::vector<std::thread> th;
        for (int p = 1; p < n; p++)
            th.emplace_back(render_part, scene, cam, params, devices, n, band, part_floats, upload, std::ref(parts[p]),
                            p, &pp[p]);
        render_part(scene, cam, params, devices, n, band, part_floats, upload, parts[0], 0, &pp[0]);
        for (auto& t : th) t.join();
    }
    for (int p = 0; p < n; p++)
        if (parts[p].rc) {
            const int rc = parts[p].rc;
            const std::string e = parts[p].err;
            drop_set(devs, *set);
            return set_error(rc, "device %d: %s", devices[p], e.c_str());
        }
    set->scene = std::move(key);
    if (prog.fn && prog.reported < prog.total) prog.fn(prog.user, prog.total, prog.total);
    // One device: its part is the frame (rows in order), nothing to gather. Several: RCCL
    // needs every device once; a repeated device, PT_GATHER=host or no RCCL: host.
    // PT_GATHER=rccl (test hook) sends a single device's part through RCCL's send-to-self.
    std::vector<int32_t> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const char* gh = hook_env("PT_GATHER");
    const bool direct = n == 1 && !(gh && (strcmp(gh, "rccl") == 0 || strcmp(gh, "host") == 0));
    std::shared_ptr<CommSet> cs;
    bool use_rccl = !direct && distinct && !(gh && strcmp(gh, "host") == 0);
    bool fell_back = false;  // RCCL was the way, but unavailable or failed: host assembly
    if (use_rccl && get_comms(devs, cs) != PT_OK) {
        note_host_gather(pt_last_error());
        use_rccl = false;
        fell_back = true;
    }
    int rc = PT_OK;
    float gather_ms = 0.0f;
    const size_t frame_floats = (size_t)H * W * 3;
    if (direct) {
        auto body = [&]() -> int {
            HIP_OK(hipSetDevice(devices[0]));
            if (out_rgb8) {
                if (const int g = grow(&set->d_rgb8, &set->rgb8_cap, frame_floats)) return g;
                const int q = rgb8_device(parts[0].ctx, parts[0].d_out, H, W, gamma, 1, set->d_rgb8);
                if (q) return q;
                HIP_OK(hipMemcpy(out_rgb8, set->d_rgb8, frame_floats, hipMemcpyDeviceToHost));
            }
            if (out_rgb) HIP_OK(hipMemcpy(out_rgb, parts[0].d_out, frame_floats * sizeof(float), hipMemcpyDeviceToHost));
            return PT_OK;
        };
        rc = body();
    } else if (use_rccl) {
        Rccl& R = rccl_table();
        hipEvent_t e0 = nullptr, e1 = nullptr;
        hipStream_t s0 = (hipStream_t)ctx_stream(parts[0].ctx);
        bool rccl_failed = false;
        auto body = [&]() -> int {
            HIP_OK(hipSetDevice(devices[0]));
            if (const int g = grow(&set->d_gather, &set->gather_cap, (size_t)n * part_floats)) return g;
            if (const int g = grow(&set->d_frame, &set->frame_cap, frame_floats)) return g;
            float* d_gather = set->d_gather;
            float* d_frame = set->d_frame;
            HIP_OK(hipEventCreate(&e0));
            HIP_OK(hipEventCreate(&e1));
            std::unique_lock<std::mutex> glock(cs->mu);  // one group at a time on these communicators
            if (cs->failed) {  // another thread's group failed meanwhile: this set is gone
                glock.unlock();
                std::shared_ptr<CommSet> fresh;
                if (get_comms(devs, fresh) != PT_OK) {
                    rccl_failed = true;
                    return set_error(PT_E_HIP, "RCCL communicators unavailable after a failed group");
                }
                cs = fresh;
                glock = std::unique_lock<std::mutex>(cs->mu);
                if (cs->failed) {
                    rccl_failed = true;
                    return set_error(PT_E_HIP, "RCCL communicators failed again");
                }
            }
            HIP_OK(hipEventRecord(e0, s0));
            // One group: part p's buffer -> device 0 (p = 0 is RCCL's send-to-self).
            std::vector<const void*> sb(n);
            std::vector<void*> rb(n);
            std::vector<hipStream_t> ss(n);
            for (int p = 0; p < n; p++) {
                sb[p] = parts[p].d_out;
                rb[p] = d_gather + (size_t)p * part_floats;
                ss[p] = (hipStream_t)ctx_stream(parts[p].ctx);
            }
            ncclResult_t r = group_gather(R, *cs, n, sb, rb, part_floats, ss, s0);
            if (r == ncclSuccess) {
                for (int p = 1; p < n && r == ncclSuccess; p++)  // the senders' streams drained too
                    if (hipStreamSynchronize(ss[p]) != hipSuccess) r = ncclUnhandledCudaError;
            }
            if (r != ncclSuccess) {
                rccl_failed = true;
                const int rc_fail = set_error(PT_E_HIP, "RCCL gather: %s", R.error_string(r));
                fail_comms(devs, cs);  // still under cs->mu: no group can be on them now
                return rc_fail;
            }
            hipLaunchKernelGGL(pt_assemble_kernel, dim3((3 * W + 255) / 256, H), dim3(256), 0, s0, d_gather, d_frame,
                               W, n, band, max_rows);
            HIP_OK(hipGetLastError());
            HIP_OK(hipEventRecord(e1, s0));
            if (out_rgb8) {
                if (const int g = grow(&set->d_rgb8, &set->rgb8_cap, frame_floats)) return g;
                const int q = rgb8_device(parts[0].ctx, d_frame, H, W, gamma, 1, set->d_rgb8);
                if (q) return q;
                HIP_OK(hipMemcpy(out_rgb8, set->d_rgb8, frame_floats, hipMemcpyDeviceToHost));
            }
            if (out_rgb) HIP_OK(hipMemcpyAsync(out_rgb, d_frame, frame_floats * sizeof(float), hipMemcpyDeviceToHost, s0));
            HIP_OK(hipStreamSynchronize(s0));
            HIP_OK(hipEventElapsedTime(&gather_ms, e0, e1));
            return PT_OK;
        };
        rc = body();
        (void)hipSetDevice(devices[0]);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (rccl_failed) {  // communicators aborted and dropped: this frame assembles on the host
            note_host_gather(pt_last_error());
            use_rccl = false;
            fell_back = true;
            rc = PT_OK;
        }
    }
    if (!direct && !use_rccl) {
        std::vector<float> host(n * part_floats);
        for (int p = 0; p < n && !rc; p++) {
            if (hipSetDevice(devices[p]) != hipSuccess ||
                hipMemcpy(host.data() + p * part_floats, parts[p].d_out, part_floats * sizeof(float),
                          hipMemcpyDeviceToHost) != hipSuccess)
                rc = set_error(PT_E_HIP, "part %d: device-to-host copy failed", p);
        }
        std::vector<float> frame;
        float* dst = out_rgb;
        if (!dst) {
            frame.resize(frame_floats);
            dst = frame.data();
        }
        for (int h = 0; h < H && !rc; h++) {
            const int kb = h / band, p = kb % n, i = (kb / n) * band + h % band;
            memcpy(dst + (size_t)h * W * 3, host.data() + p * part_floats + (size_t)i * W * 3,
                   (size_t)W * 3 * sizeof(float));
        }
        if (!rc && out_rgb8) rc = pt_image_to_rgb8(dst, W, H, gamma, out_rgb8);
    }
    if (!rc && stats) {
        memset(stats, 0, sizeof(*stats));
        for (int p = 0; p < n; p++) {
            stats->rays += parts[p].st.rays;
            stats->paths += parts[p].st.paths;
            stats->runaway += parts[p].st.runaway;
            stats->kernel_ms = std::max(stats->kernel_ms, parts[p].st.kernel_ms);
            stats->reduce_ms = std::max(stats->reduce_ms, parts[p].st.reduce_ms);
            stats->trace_launches += parts[p].st.trace_launches;
            stats->kernel_path = parts[p].st.kernel_path;
            stats->device_kernel_ms[p] = parts[p].st.kernel_ms;
            stats->device_render_ms[p] = parts[p].render_ms;
            stats->device_rays[p] = parts[p].st.rays;
        }
        stats->n_devices = n;
        stats->rows = H;
        stats->gather_ms = gather_ms;
        stats->gather_path = direct     ? PT_GATHER_NONE
                             : use_rccl  ? PT_GATHER_RCCL
                             : fell_back ? PT_GATHER_HOST_FALLBACK
                                         : PT_GATHER_HOST;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    if (rc || !cached) {
        drop_set(devs, *set);
    } else {
        for (int p = 0; p < n; p++) (void)ctx_release_slabs(parts[p].ctx);
    }
    return rc;
}

}  // namespace
}  // namespace pt

extern "C" {

int pt_render_f32_devices(const pt_scene* scene, const pt_camera* cam, const pt_params* params,
                          const int32_t* devices, int32_t n_devices, float* out_rgb, pt_stats* stats) {
    if (!out_rgb) return pt::set_error(PT_E_ARG, "pt_render_f32_devices: out_rgb is NULL");
    return pt::render_devices(scene, cam, params, devices, n_devices, out_rgb, nullptr, 2.2f, stats);
}

int pt_render_rgb8_devices(const pt_scene* scene, const pt_camera* cam, const pt_params* params,
                           const int32_t* devices, int32_t n_devices, float gamma, uint8_t* rgb8, pt_stats* stats) {
    if (!rgb8) return pt::set_error(PT_E_ARG, "pt_render_rgb8_devices: rgb8 is NULL");
    return pt::render_devices(scene, cam, params, devices, n_devices, nullptr, rgb8, gamma, stats);
}

void pt_devices_release(void) {
    using namespace pt;
    std::map<std::vector<int32_t>, std::shared_ptr<DevSet>> sets;
    {
        std::lock_guard<std::mutex> g(g_dev_sets_mu);
        sets.swap(g_dev_sets);
    }
    for (auto& kv : sets) {
        std::lock_guard<std::mutex> l(kv.second->mu);  // after any render still running on it
        drop_set(kv.first, *kv.second);
    }
}

// Test hook: process-wide counters (pt_hip_debug.h).
int64_t pt_debug_counter(int32_t which) {
    using namespace pt;
    if (which == 0 || which == 1) return kernel_counter(which);
    if (which == 2) {
        std::lock_guard<std::mutex> g(g_dev_sets_mu);
        int64_t live = 0;
        for (auto& kv : g_dev_sets) {
            std::lock_guard<std::mutex> l(kv.second->mu);
            live += kv.second->parts.empty() ? 0 : 1;
        }
        return live;
    }
    if (which == 3) return g_upload_skips.load();
    return set_error(PT_E_ARG, "pt_debug_counter: bad counter %d", which);
}

}  // extern "C"

// ---- test hook: the communicator cache's failure handling with a fake RCCL table
namespace pt {
namespace {
struct FakeRccl {
    int fail_step = -1;  // which call fails: 0 init, 1 group start, 2 send, 3 recv, 4 group end, -1 none
    int64_t created = 0, aborted = 0;
    std::vector<char> live;  // per fake communicator handle: 1 while neither aborted nor destroyed
};
FakeRccl* g_fake = nullptr;
ncclComm_t fake_handle(size_t i) { return reinterpret_cast<ncclComm_t>((uintptr_t)(i + 1) * 16); }
ncclResult_t fake_init_all(ncclComm_t* comms, int n, const int*) {
    for (int i = 0; i < n; i++) {  // a partial init: the first communicators exist when it fails
        if (g_fake->fail_step == 0 && i == n / 2) return ncclSystemError;
        g_fake->live.push_back(1);
        comms[i] = fake_handle(g_fake->live.size() - 1);
        g_fake->created++;
    }
    return ncclSuccess;
}
ncclResult_t fake_group_start() { return g_fake->fail_step == 1 ? ncclSystemError : ncclSuccess; }
ncclResult_t fake_group_end() { return g_fake->fail_step == 4 ? ncclSystemError : ncclSuccess; }
ncclResult_t fake_send(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) {
    return g_fake->fail_step == 2 ? ncclSystemError : ncclSuccess;
}
ncclResult_t fake_recv(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) {
    return g_fake->fail_step == 3 ? ncclSystemError : ncclSuccess;
}
const char* fake_error_string(ncclResult_t) { return "injected failure"; }
ncclResult_t fake_abort(ncclComm_t c) {
    const size_t i = (size_t)(reinterpret_cast<uintptr_t>(c) / 16) - 1;
    if (i < g_fake->live.size() && g_fake->live[i]) {
        g_fake->live[i] = 0;
        g_fake->aborted++;
    }
    return ncclSuccess;
}
}  // namespace
}  // namespace pt

extern "C" {

// Test hook (no device needed): the RCCL communicator cache of pt_render_*_devices driven
// through a fake RCCL table whose call `fail_step` fails (0 ncclCommInitAll, 1
// ncclGroupStart, 2 ncclSend, 3 ncclRecv, 4 ncclGroupEnd, -1 none). One gather over
// n_devices fake devices, then a second one. out[0] communicators created, out[1] aborted,
// out[2] communicators still live, out[3] cache entries for the list after the first gather,
// out[4] 1 if the second gather got a different set (a failed set is never reused), out[5]
// the first gather's result (0 = success). The real cache and table are restored.
int pt_debug_rccl_failover(int32_t n_devices, int32_t fail_step, int64_t* out) {
    using namespace pt;
    if (!out || n_devices < 1 || n_devices > PT_MAX_DEVICES || fail_step < -1 || fail_step > 4)
        return set_error(PT_E_ARG, "pt_debug_rccl_failover: bad argument");
    std::vector<int32_t> devs;
    for (int i = 0; i < n_devices; i++) devs.push_back(1000 + i);  // device ids no real list uses
    FakeRccl fake;
    fake.fail_step = fail_step;
    Rccl table;
    table.ok = true;
    table.comm_init_all = fake_init_all;
    table.group_start = fake_group_start;
    table.group_end = fake_group_end;
    table.send = fake_send;
    table.recv = fake_recv;
    table.error_string = fake_error_string;
    table.comm_abort = fake_abort;
    g_fake = &fake;
    g_rccl_fake = &table;
    auto gather = [&](std::shared_ptr<CommSet>& cs) -> int {
        if (get_comms(devs, cs) != PT_OK) return 1;
        std::lock_guard<std::mutex> glock(cs->mu);
        std::vector<const void*> sb(n_devices, nullptr);
        std::vector<void*> rb(n_devices, nullptr);
        std::vector<hipStream_t> ss(n_devices, nullptr);
        if (group_gather(table, *cs, n_devices, sb, rb, 0, ss, nullptr) != ncclSuccess) {
            fail_comms(devs, cs);
            return 2;
        }
        return 0;
    };
    std::shared_ptr<CommSet> first, second;
    const int r1 = gather(first);
    int64_t entries = 0;
    {
        std::lock_guard<std::mutex> lock(g_comm_mu);
        entries = (int64_t)g_comms.count(devs);
    }
    fake.fail_step = -1;
    const int r2 = gather(second);
    int64_t live = 0;
    for (char l : fake.live) live += l;
    out[0] = fake.created;
    out[1] = fake.aborted;
    out[2] = live;
    out[3] = entries;
    out[4] = (r2 == 0 && second && second != first) ? 1 : 0;
    out[5] = r1;
    {  // leave no fake communicator in the real cache
        std::lock_guard<std::mutex> lock(g_comm_mu);
        g_comms.erase(devs);
    }
    g_rccl_fake = nullptr;
    g_fake = nullptr;
    return PT_OK;
}

}  // extern "C"
