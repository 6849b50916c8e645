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
#include <stdio.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pt_internal.h"

namespace pt {

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
        x->ok = x->comm_init_all && x->group_start && x->group_end && x->send && x->recv && x->error_string;
        if (!x->ok) x->why = "librccl lacks a needed symbol";
        return x;
    }();
    return *r;
}

// One communicator per device of a device list, created once per process (init costs
// hundreds of ms) and kept: RCCL communicators are not torn down at exit. Each set has
// its own mutex, held from ncclGroupStart until the gather's stream is drained: two host
// threads rendering over the same device list must not interleave groups on the same
// communicators. A set whose group failed is dropped from the cache (the next call
// makes a fresh one) and that call assembles the frame on the host.
struct CommSet {
    std::vector<ncclComm_t> comms;
    std::mutex mu;
};
std::mutex g_comm_mu;
std::map<std::vector<int32_t>, std::shared_ptr<CommSet>> g_comms;

int get_comms(const std::vector<int32_t>& devs, std::shared_ptr<CommSet>& out) {
    Rccl& R = rccl();
    if (!R.ok) return set_error(PT_E_HIP, "%s", R.why.c_str());
    std::lock_guard<std::mutex> lock(g_comm_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        auto cs = std::make_shared<CommSet>();
        cs->comms.assign(devs.size(), nullptr);
        // RCCL prints its version banner to stdout at init; the drop-in's stdout is the
        // reference's console contract (render.h:79-101), so the banner goes to stderr
        fflush(stdout);
        const int saved = dup(1);
        if (saved >= 0) dup2(2, 1);
        const ncclResult_t r = R.comm_init_all(cs->comms.data(), (int)devs.size(), devs.data());
        fflush(stdout);
        if (saved >= 0) {
            dup2(saved, 1);
            close(saved);
        }
        if (r != ncclSuccess) return set_error(PT_E_HIP, "ncclCommInitAll: %s", R.error_string(r));
        it = g_comms.emplace(devs, std::move(cs)).first;
    }
    out = it->second;
    return PT_OK;
}

void drop_comms(const std::vector<int32_t>& devs, const std::shared_ptr<CommSet>& cs) {
    std::lock_guard<std::mutex> lock(g_comm_mu);
    auto it = g_comms.find(devs);
    if (it != g_comms.end() && it->second == cs) g_comms.erase(it);
}

// Why a gather over distinct devices went through the host, once per process on stderr.
void note_host_gather(const std::string& why) {
    static std::once_flag once;
    std::call_once(once, [&] {
        fprintf(stderr, "[libpt_hip] RCCL gather unavailable (%s); parts assembled on the host\n", why.c_str());
    });
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
// buffer has the gather's common size).
struct Part {
    pt_ctx* ctx = nullptr;
    float* d_out = nullptr;
    pt_stats st{};
    int rc = PT_OK;
    std::string err;
    double render_ms = 0.0;
};

// Render part p of the partition on devices[p] into parts[p].d_out (device memory).
void render_part(const pt_scene* scene, const pt_camera* cam, const pt_params* params, const int32_t* devices,
                 int n, int band, size_t part_floats, Part& P, int p, PartProgress* pp) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc = pt_ctx_create(devices[p], &P.ctx);
    if (!rc) rc = pt_ctx_set_scene(P.ctx, scene);
    if (!rc && hipSetDevice(devices[p]) != hipSuccess) rc = set_error(PT_E_HIP, "hipSetDevice failed");
    if (!rc && hipMalloc((void**)&P.d_out, std::max<size_t>(part_floats, 1) * sizeof(float)) != hipSuccess)
        rc = set_error(PT_E_HIP, "hipMalloc of the part buffer failed");
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
    for (size_t p = 0; p < parts.size(); p++) {
        if (parts[p].d_out) {
            (void)hipSetDevice(devices[p]);
            (void)hipFree(parts[p].d_out);
        }
        if (parts[p].ctx) pt_ctx_destroy(parts[p].ctx);
    }
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
    const int n = n_devices, band = params->band_rows > 0 ? params->band_rows : 8;
    int max_rows = 0;
    for (int p = 0; p < n; p++) max_rows = std::max(max_rows, (int)pt_part_rows(H, p, n, band));
    const size_t part_floats = (size_t)max_rows * W * 3;
    std::vector<Part> parts(n);
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
            th.emplace_back(render_part, scene, cam, params, devices, n, band, part_floats, std::ref(parts[p]), p,
                            &pp[p]);
        render_part(scene, cam, params, devices, n, band, part_floats, parts[0], 0, &pp[0]);
        for (auto& t : th) t.join();
    }
    for (int p = 0; p < n; p++)
        if (parts[p].rc) {
            const int rc = parts[p].rc;
            const std::string e = parts[p].err;
            release(parts, devices);
            return set_error(rc, "device %d: %s", devices[p], e.c_str());
        }
    if (prog.fn && prog.reported < prog.total) prog.fn(prog.user, prog.total, prog.total);
    // One device: its part is the frame (rows in order), nothing to gather. Several: RCCL
    // needs every device once; a repeated device, PT_GATHER=host or no RCCL: host.
    // PT_GATHER=rccl (test hook) sends a single device's part through RCCL's send-to-self.
    std::vector<int32_t> devs(devices, devices + n);
    std::vector<int32_t> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const char* gh = hook_env("PT_GATHER");
    const bool direct = n == 1 && !(gh && (strcmp(gh, "rccl") == 0 || strcmp(gh, "host") == 0));
    std::shared_ptr<CommSet> cs;
    bool use_rccl = !direct && distinct && !(gh && strcmp(gh, "host") == 0);
    if (use_rccl && get_comms(devs, cs) != PT_OK) {
        note_host_gather(pt_last_error());
        use_rccl = false;
    }
    int rc = PT_OK;
    float gather_ms = 0.0f;
    const size_t frame_floats = (size_t)H * W * 3;
    if (direct) {
        uint8_t* d_rgb8 = nullptr;
        auto body = [&]() -> int {
            HIP_OK(hipSetDevice(devices[0]));
            if (out_rgb8) {
                HIP_OK(hipMalloc((void**)&d_rgb8, std::max<size_t>(frame_floats, 1)));
                const int q = rgb8_device(parts[0].ctx, parts[0].d_out, H, W, gamma, 1, d_rgb8);
                if (q) return q;
                HIP_OK(hipMemcpy(out_rgb8, d_rgb8, frame_floats, hipMemcpyDeviceToHost));
            }
            if (out_rgb) HIP_OK(hipMemcpy(out_rgb, parts[0].d_out, frame_floats * sizeof(float), hipMemcpyDeviceToHost));
            return PT_OK;
        };
        rc = body();
        if (d_rgb8) (void)hipFree(d_rgb8);
    } else if (use_rccl) {
        Rccl& R = rccl();
        float* d_gather = nullptr;
        float* d_frame = nullptr;
        uint8_t* d_rgb8 = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        hipStream_t s0 = (hipStream_t)ctx_stream(parts[0].ctx);
        bool rccl_failed = false;
        auto body = [&]() -> int {
            HIP_OK(hipSetDevice(devices[0]));
            HIP_OK(hipMalloc((void**)&d_gather, std::max<size_t>((size_t)n * part_floats, 1) * sizeof(float)));
            HIP_OK(hipMalloc((void**)&d_frame, frame_floats * sizeof(float)));
            HIP_OK(hipEventCreate(&e0));
            HIP_OK(hipEventCreate(&e1));
            std::lock_guard<std::mutex> glock(cs->mu);  // one group at a time on these communicators
            HIP_OK(hipEventRecord(e0, s0));
            // One group: part p's buffer -> device 0 (p = 0 is RCCL's send-to-self).
            ncclResult_t r = R.group_start();
            for (int p = 0; p < n && r == ncclSuccess; p++)
                r = R.send(parts[p].d_out, part_floats, ncclFloat32, 0, cs->comms[p],
                           (hipStream_t)ctx_stream(parts[p].ctx));
            for (int p = 0; p < n && r == ncclSuccess; p++)
                r = R.recv(d_gather + (size_t)p * part_floats, part_floats, ncclFloat32, p, cs->comms[0], s0);
            const ncclResult_t re = R.group_end();
            if (r == ncclSuccess) r = re;
            if (r == ncclSuccess) {
                for (int p = 1; p < n && r == ncclSuccess; p++)  // the senders' streams drained too
                    if (hipStreamSynchronize((hipStream_t)ctx_stream(parts[p].ctx)) != hipSuccess) r = ncclUnhandledCudaError;
            }
            if (r != ncclSuccess) {
                rccl_failed = true;
                return set_error(PT_E_HIP, "RCCL gather: %s", R.error_string(r));
            }
            hipLaunchKernelGGL(pt_assemble_kernel, dim3((3 * W + 255) / 256, H), dim3(256), 0, s0, d_gather, d_frame,
                               W, n, band, max_rows);
            HIP_OK(hipGetLastError());
            HIP_OK(hipEventRecord(e1, s0));
            if (out_rgb8) {
                HIP_OK(hipMalloc((void**)&d_rgb8, std::max<size_t>(frame_floats, 1)));
                const int q = rgb8_device(parts[0].ctx, d_frame, H, W, gamma, 1, d_rgb8);
                if (q) return q;
                HIP_OK(hipMemcpy(out_rgb8, d_rgb8, frame_floats, hipMemcpyDeviceToHost));
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
        if (d_gather) (void)hipFree(d_gather);
        if (d_frame) (void)hipFree(d_frame);
        if (d_rgb8) (void)hipFree(d_rgb8);
        if (rccl_failed) {  // drop the communicators, assemble this frame on the host instead
            note_host_gather(pt_last_error());
            drop_comms(devs, cs);
            use_rccl = false;
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
        stats->gather_path = direct ? PT_GATHER_NONE : use_rccl ? PT_GATHER_RCCL : PT_GATHER_HOST;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    release(parts, devices);
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

}  // extern "C"
