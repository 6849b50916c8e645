/*
 * pt_hip_debug.h — test and tuning hooks of libpt_hip.so, kept apart from the drop-in
 * boundary (include/pt_hip.h). Nothing a reference-side binding needs is declared here;
 * the tests (tests/test_capi.py, tests/test_gpu_parity.py, tests/test_math.py) call these
 * through ctypes. Every symbol is exported by libpt_hip.so.
 */
#ifndef PT_HIP_DEBUG_H
#define PT_HIP_DEBUG_H

#include "pt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Run the device copies of the path's math primitives on `device`:
 * which = 0: acosf(in[i]) -> out[i]
 *         1: sincosf(in[i]) -> out[2i] = sin, out[2i+1] = cos
 *         2: BRDF sample; in[9i..9i+8] = {lcg state (bits), material type (bits),
 *            roughness, d.xyz, n.xyz} -> out[4i..4i+3] = {dir.xyz, state after (bits)} */
int pt_debug_math(int device, int which, const float* in, int n, float* out);
/* Exhaustive check of a fast device sequence against its IEEE-exact counterpart over
 * every float bit pattern in [lo_bits, hi_bits] (NaN inputs skipped), on `device`:
 * which = 0: rcp_exact(x) vs 1.0f / x;  1: sqrt_exact(x) vs sqrtf(x);
 *         2: acosf fast vs restatement;  3: sincosf fast vs restatement (pt_math.h);
 *         4: div_by_rcp(x, b, RN(1/b)) vs x / b for a hashed divisor b per input x.
 * *mismatches = number of differing results, *first_bad = lowest differing input bits
 * (0xffffffff if none). */
int pt_debug_sweep(int device, int which, uint32_t lo_bits, uint32_t hi_bits, uint64_t* mismatches,
                   uint32_t* first_bad);
/* The device quantiser (pt_ctx_render_rgb8's second half) on a host image: rgb8 = top
 * row first, as pt_image_to_rgb8. */
int pt_debug_rgb8(int device, const float* linear_rgb, int32_t res_x, int32_t res_y, float gamma, uint8_t* rgb8);
/* Test hook, no device needed: the multi-device gather's communicator cache driven through a
 * fake RCCL table whose call `fail_step` fails (0 init, 1 group start, 2 send, 3 recv,
 * 4 group end, -1 none); out[6] = {created, aborted, still live, cache entries after the
 * first gather, second gather got a fresh set, first gather's result}. */
int pt_debug_rccl_failover(int32_t n_devices, int32_t fail_step, int64_t* out);
/* Rebuild the wide tree (width 4 or 8) of `scene` and check its invariants exactly on the
 * host: quantised child boxes contain the reference's boxes, child links, triangle ranks
 * and exact leaf boxes, every triangle stored once. Returns the violation count (0 = ok). */
int pt_debug_wide_verify(const pt_scene* scene, int32_t width);
/* Test hook, no device needed: *hash = FNV-1a 64 of every array and scalar the scene packing
 * produces (device layout, flat leaves, wide tree), to check that the packing's thread
 * schedule (PT_PACK_THREADS) leaves its output bit-identical. */
int pt_debug_pack_hash(const pt_scene* scene, uint64_t* hash);
/* Generate (into src_out, if non-NULL) and compile the hipRTC scene-specialised flat
 * kernel for `scene` without touching a device. Returns the code-object size (> 0). */
int pt_rtc_check(const pt_scene* scene, char* src_out, size_t cap);
/* Test hook, no device needed: start the scene kernel's compile in the background, as
 * pt_ctx_set_scene does, and return at once (1: a compile is running, 0: already done). */
int pt_debug_rtc_start(const pt_scene* scene);
/* Test hook, no device needed: the scene kernel's code-object caches (an on-disk cache
 * under $PT_RTC_CACHE_DIR, $XDG_CACHE_HOME/pathtracer-amd/rtc or ~/.cache/pathtracer-amd/rtc,
 * off with PT_RTC_CACHE=0; entries verified by sha256 on load). op 0 forgets this process's
 * compiles, 1 disk hits, 2 rejected entries, 3 compiles so far, 4 the last compile's wall time
 * in microseconds, 5 compiles done by the compile server (bin/pt_rtc_server). */
int64_t pt_debug_rtc_cache(int32_t op);

/* Test hook: how a context's scene is rendered. out[0] = 1 if the scene kernel unwinds with
 * pre-doubled albedo (the host's radiance bound passed, pt_kernel.hip: albedo_x2_ok), out[1] =
 * 1 if the scene holds a SPECULAR material, out[2] = 1 if a hipRTC scene kernel was requested
 * for the scene, out[3] = wide nodes (0 = no wide tree), out[4] = 1 if every bounce material is
 * dark (emission +0, finite albedo: finish_path skips the unwinding of +0 paths). */
int pt_debug_ctx_flags(const pt_ctx* ctx, int32_t out[5]);
/* Test hook, no device needed: 1 if `scene` passes the dark-path gate (every non-emitting
 * triangle: emission +0, finite albedo, a unit-length shading normal, SPECULAR roughness
 * |r| <= 1.15 so that cos theta is finite; pt_kernel.hip scene_dark), 0 if not, < 0 on error. */
int pt_debug_scene_dark(const pt_scene* scene);
/* Test hook: process-wide counters. which = 0: contexts created (pt_ctx_create), 1: scene
 * uploads (pt_ctx_set_scene), 2: cached multi-device context sets live, 3: uploads skipped
 * because a cached context already held the same scene. */
int64_t pt_debug_counter(int32_t which);

#ifdef __cplusplus
}
#endif
#endif /* PT_HIP_DEBUG_H */
