#!/usr/bin/env python3
"""Benchmark: Mray/s of the gfx950 trace kernel on the README headline config.

Workload (BASELINE.json configs[1]): Cornell box (examples/cornell_box.cc,
32 triangles) at 1024x1024, 10,000 spp, depth 5 — one step = one full frame.
With N GPUs (torchrun, one process per GPU) the frame's rows are dealt to the
ranks row by row (1-row bands; the reference's tile loop, render.h:128-139, made
static) and gathered to rank 0 over RCCL; total work is fixed ("strong").
--scene / --spp / --res / --depth / --rough select the other configs.

value = rays traced by all ranks / max-over-ranks wall time of the K timed
steps (rays = BVH::intersect calls, every segment incl. misses and emitter
hits).

Rooflines:
  roofline       — the binding one, VALU main-port issue: SQ_ACTIVE_INST_VALU minus the
                   second port's SQ_ACTIVE_INST_VALU2 per ray of THIS kernel build (rocprofv3
                   PMC passes, profiles/pmc/<workload>.json, keyed to the sha256 of the
                   kernel sources; null when the key does not match) x rays per launch / the
                   live average launch time (HIP events), against 256 CUs x 4 SIMDs x 2.4 GHz
                   / 4 cycles per main-port slot (calibrated).
  hbm_algorithmic — SURVEY.md §8(d)'s reference-layout bytes per ray (985 B for
                   Cornell d5) / launch time, against 8 TB/s. The scene lives in LDS
                   and hipRTC constants, so this is not HBM traffic and exceeds 1.
  hbm_measured   — FETCH_SIZE x 2 + WRITE_SIZE per ray from the same keyed PMC pass.
The CPU baseline is the unmodified reference binary (oracle/_ref/pt_ref) on one host
core over a bounded sample of the same workload, its image compared bit for bit.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scene S] [--spp S] [--res R] [--depth D]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))

# Algorithmic bytes per ray in the reference layout: 40 B per node visit (BVHNode),
# 40 B per triangle test (36 B vertices + 4 B tri_idx), 32 B Material per hit.
# Per-ray counts from the CPU oracle at the pinned seeding.
B_RAY = {("cornell", 5): 985.0, ("cornell", 3): 957.0, ("cornell", 8): 1004.0, ("mcornell", 5): 1100.0,
         ("sphere", 5): 1489.0}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# VALU main-port issue peak (calibrated with tools/valu_ubench under rocprofv3,
# profiles/archive/r03_valu_calibration): a wave64 VALU instruction occupies the SIMD's main port for 4
# cycles (v_fma_f32 at full occupancy: 3.9-4.1 cycles; SQ_INSTS_VALU = exactly one count per
# wave-instruction); simple f32 add/sub/mul and integer add/and/mov may issue on a second port
# instead (SQ_ACTIVE_INST_VALU2), transcendentals take two slots (8 cycles).
VALU_PEAK_G = 256 * 4 * 2.4 / 4  # G main-port slots/s at 2.4 GHz
README_MRAYS = 331.0  # BASELINE.md §1 derived rate of the published 112 s Cornell frame
# Sources whose bytes decide the kernel a PMC pass measured (device code, packing, launch).
KERNEL_SOURCES = ["pathtracer-cpp_amd/csrc/pt_trace.h", "pathtracer-cpp_amd/csrc/pt_kernel.hip",
                  "pathtracer-cpp_amd/csrc/pt_math.h", "pathtracer-cpp_amd/csrc/pt_host.cpp",
                  "pathtracer-cpp_amd/csrc/pt_internal.h", "include/pt_hip.h", "pathtracer-cpp_amd/Makefile",
                  "pathtracer-cpp_amd/csrc/pt_flat_fast.hip"]


def kernel_key() -> str:
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--spp", type=int, default=10000)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--scene", choices=["cornell", "mcornell", "sphere"], default="cornell",
                    help="cornell (configs 1/2/5), mcornell (config 3, --rough), sphere (config 4 mesh)")
    ap.add_argument("--rough", type=float, default=0.3, help="modified Cornell roughness")
    ap.add_argument("--band", type=int, default=1, help="rows per band of the row partition (1: best balance)")
    ap.add_argument("--part", default="", help="P/N: one GPU renders only part P of an N-way row partition "
                                              "(a rank's share at --gpus N, timed alone)")
    ap.add_argument("--per-item", type=int, default=0, help="samples per work item (0 = library default)")
    ap.add_argument("--batch", type=int, default=0, help="samples per accumulation batch (0 = auto)")
    ap.add_argument("--cpu-spp", type=int, default=0,
                    help="spp of the bounded CPU-baseline sample (0: per scene, ~10-30 s of CPU work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (cold setup + render + D2H) pass")
    ap.add_argument("--e2e-only", action="store_true",
                    help="only the end-to-end pass, its JSON on stdout (the warm-cache run bench.py starts itself)")
    return ap.parse_args()


def host_info() -> dict:
    model = platform.processor() or "?"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable}


def cpu_baseline(a, scene, bvh, gpu_renderer, cam):
    """Reference render_cpu loop (unmodified, 1 core) on a bounded sample of the same
    workload: every pixel of the frame at `spp` samples (config 1: the whole config).
    Rays come from the GPU render of the same sample, whose image must be bit-identical.
    The 99k-triangle mesh loads the fast builder's tree (bit-identical to BVH::build by
    its sha256, tests/test_capi.py) instead of re-running the reference's 380 s build."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    W, H = scene.camera.res
    spp = a.cpu_spp or {"cornell": 16 if a.depth <= 5 else 8, "mcornell": 8, "sphere": 8}[a.scene]
    spp = min(spp, a.spp)
    gpu_img, st = gpu_renderer.render(cam, spp, a.depth)
    info = host_info()
    if O.ref_available():
        kind = "reference"
        with tempfile.TemporaryDirectory() as td:
            sp = os.path.join(td, "s.ptscene")
            with open(sp, "w") as f:
                f.write(scene.to_ptscene())
            out = os.path.join(td, "o.f32")
            cmd = [O.REF_BIN, "--scene", sp, "--spp", str(spp), "--depth", str(a.depth), "--out", out]
            if a.scene == "sphere":
                bp = os.path.join(td, "bvh.bin")
                with open(bp, "wb") as f:
                    np.array([len(bvh.nodes), len(bvh.tri_idx)], dtype=np.int32).tofile(f)
                    np.ascontiguousarray(bvh.nodes).tofile(f)
                    np.ascontiguousarray(bvh.tri_idx, dtype=np.int32).tofile(f)
                cmd += ["--load-bvh", bp]
            try:
                if subprocess.run(["taskset", "-c", "0", "true"]).returncode == 0:
                    cmd = ["taskset", "-c", "0"] + cmd
            except FileNotFoundError:
                pass
            r = subprocess.run(cmd, check=True, capture_output=True, text=True)
            meta = json.loads(r.stdout.strip().splitlines()[-1])
            secs = meta["render_s"]
            ref = np.fromfile(out, dtype=np.float32).reshape(H, W, 3)
    else:
        kind = "port"
        t0 = time.perf_counter()
        ref, _ = O.render(scene, spp, a.depth)
        secs = time.perf_counter() - t0
    same = bool(np.array_equal(ref.view(np.uint32), gpu_img.view(np.uint32)))
    return {"value": st["rays"] / secs / 1e6, "unit": "Mray/s", "cores": 1, "kind": kind,
            "sample": f"{scene.name} {W}x{H}, {spp} spp, depth {a.depth}: {st['rays']} rays in {secs:.2f} s "
                      f"(single thread; image bit-identical to GPU: {same})",
            "seconds": secs, "bitexact_vs_gpu": same, **info,
            "full_config_extrapolated_s": secs * a.spp / spp}


def load_pmc(workload: str):
    path = os.path.join(ROOT, "profiles", "pmc", workload + ".json")
    if not os.path.exists(path):
        return None, f"no PMC pass for {workload}"
    with open(path) as f:
        pm = json.load(f)
    key = kernel_key()
    if pm.get("key") != key:
        return None, f"PMC pass {pm.get('source')} is for kernel key {pm.get('key')}, this build is {key}"
    return pm, pm.get("source")


def warm_e2e(a, rtc_dir):
    """The end-to-end pass again in a fresh process whose code-object cache holds this
    scene's kernel (written by the cold pass): what a second run of a drop-in program pays.
    Context, scene setup and the frame are in it; the device initialisation is reported
    beside it, as in the cold pass."""
    args = [sys.executable, os.path.abspath(__file__), "--e2e-only", "--scene", a.scene, "--spp", str(a.spp),
            "--res", str(a.res), "--depth", str(a.depth), "--rough", str(a.rough), "--band", str(a.band),
            "--batch", str(a.batch), "--per-item", str(a.per_item)]
    env = dict(os.environ, PT_RTC_CACHE_DIR=rtc_dir)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    try:
        r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=600)
        return json.loads(r.stdout.strip().splitlines()[-1])["end_to_end"]
    except (subprocess.SubprocessError, ValueError, IndexError, KeyError) as e:
        return {"error": f"{type(e).__name__}: {e}"}


def make_scene(a):
    from ptamd import scenes
    if a.scene == "cornell":
        return scenes.cornell((a.res, a.res))
    if a.scene == "mcornell":
        return scenes.modified_cornell(float(np.float32(a.rough)), (a.res, a.res))
    return scenes.sphere_in_cornell(223, (a.res, a.res))


def die(msg: str) -> None:
    print(f"[bench] error: {msg}", file=sys.stderr, flush=True)
    sys.exit(2)


def main():
    """Entry: the world comes from a launcher (torchrun: WORLD_SIZE, which must equal
    --gpus) or, without one, --gpus N > 1 spawns N ranks here (ptamd.dist.spawn_ranks,
    the environment torchrun would set) before this process touches a GPU. Fewer visible
    GPUs than N is an error, never a silent 1-GPU run."""
    a = parse()
    if a.gpus < 1:
        die(f"--gpus {a.gpus}: need at least 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != a.gpus:
            die(f"the launcher started WORLD_SIZE={env_world} ranks but --gpus is {a.gpus}")
        run_rank(a, int(os.environ.get("RANK", "0")), a.gpus, int(os.environ.get("LOCAL_RANK", "0")),
                 os.environ.get("PT_LAUNCHER", "torchrun"), None)
        return
    import torch  # device_count() does not initialise the GPU; nothing else here touches it
    visible = torch.cuda.device_count()
    if (a.gpus == 1 or os.environ.get("PT_BENCH_BACKEND", "nccl") == "nccl") and visible < a.gpus:
        die(f"--gpus {a.gpus} but {visible} GPU(s) visible: refusing to time fewer GPUs than requested")
    if a.gpus == 1:
        run_rank(a, 0, 1, 0, "none", None)
        return
    from ptamd import dist as pdist
    with tempfile.TemporaryDirectory() as td:
        res = os.path.join(td, "result.json")
        pdist.spawn_ranks(spawned_rank, a.gpus, (vars(a), res))
        with open(res) as f:
            line = f.read()
    os.write(JSON_FD, line.encode())


def spawned_rank(rank: int, world: int, args: dict, result_path: str) -> None:
    """One rank started by main()'s spawn (the environment is torchrun's)."""
    run_rank(argparse.Namespace(**args), rank, world, rank, "spawn", result_path)


def run_rank(a, rank: int, world: int, local: int, launcher: str, result_path):
    """The benchmark body of one rank. Rank 0 writes the JSON line (to result_path when the
    ranks were spawned by main(), else to stdout)."""
    import torch
    dist = None
    # PT_BENCH_BACKEND=gloo (rehearsal only): the N>1 path with the collectives on gloo and
    # ranks sharing the visible GPUs (rank r on GPU r mod count), e.g. 2 ranks on a 1-GPU box.
    backend = os.environ.get("PT_BENCH_BACKEND", "nccl")
    dev_index = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
    if world > 1:
        import torch.distributed as dist
        if dev_index >= torch.cuda.device_count():
            die(f"rank {rank}: local rank {local} has no GPU ({torch.cuda.device_count()} visible)")
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world or dist.get_rank() != rank:
            die(f"process group has world {dist.get_world_size()} rank {dist.get_rank()}, expected {world} / {rank}")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", dev_index if world > 1 else 0)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")  # where the small all_reduces run
    # The HIP runtime's device initialisation (HSA agents, queues: 0.08-0.4 s on a fresh box,
    # scripts/ctx_timing.py) is process start-up, like importing torch: done and timed here and
    # reported beside the end-to-end figure (end_to_end.device_init_s, value_with_device_init).
    t0 = time.perf_counter()
    torch.zeros(1, device=dev).sum().item()
    t_dev_init = time.perf_counter() - t0

    import ptamd
    from ptamd import dist as pdist

    def log(msg):
        if rank == 0:
            print(msg, file=sys.stderr, flush=True)

    # ---- setup, timed cold: BVH::build (fast builder), context, scene packing + wide
    # tree + H2D, hipRTC specialisation started (render.h:115-123's build + GL upload).
    # Cold means no code-object cache either: the scene kernel's on-disk cache points at a
    # fresh directory for this process (the warm-cache pass, a child process, reuses it).
    rtc_dir = None
    if not a.e2e_only:
        rtc_dir = tempfile.mkdtemp(prefix="pt_bench_rtc_")
        os.environ["PT_RTC_CACHE_DIR"] = rtc_dir
    scene = make_scene(a)
    scene_uses_rtc = a.scene in ("cornell", "mcornell")
    bvh = ptamd.BVH.from_scene(scene)
    t0 = time.perf_counter()
    bvh.build()
    t_build = time.perf_counter() - t0
    cam = ptamd.Camera.from_spec(scene.camera)
    t0 = time.perf_counter()
    r = ptamd.Renderer(dev.index)
    t_ctx = time.perf_counter() - t0
    r.set_scene(bvh)
    torch.cuda.synchronize()
    t_scene = time.perf_counter() - t0
    W, H = a.res, a.res
    part_index, part_count = rank, world
    if a.part:
        if world > 1:
            die("--part emulates one rank's share on one GPU; it does not combine with --gpus > 1")
        part_index, part_count = (int(v) for v in a.part.split("/"))
        if not 0 <= part_index < part_count:
            die(f"--part {a.part}: need 0 <= P < N")
    rows = r.part_rows(H, part_index, part_count, a.band)
    max_rows = max(max(r.part_rows(H, p, world, a.band) for p in range(world)), rows)
    part = torch.empty(max(max_rows, 1) * W * 3, dtype=torch.float32, device=dev)

    def step():
        """One frame: this rank's rows (the render call returns once its stream is drained),
        then the gather to rank 0. st gets the host wall time of each: render_s, gather_s."""
        t_a = time.perf_counter()
        _, st = r.render(cam, a.spp, a.depth, part_index=part_index, part_count=part_count, band_rows=a.band,
                         out=part[: rows * W * 3], batch_spp=a.batch, samples_per_item=a.per_item)
        t_b = time.perf_counter()
        frame = None
        if world > 1:
            frame = pdist.gather_frame_to(part[: rows * W * 3], H, W, rank, world, a.band, dst=0)  # RCCL over xGMI
            torch.cuda.synchronize()
        st["render_s"], st["gather_s"] = t_b - t_a, time.perf_counter() - t_b
        return st, frame

    # ---- end to end, cold: BVH build + scene setup (pack, wide tree, H2D; the hipRTC
    # compile starts in the background) as timed above, plus the first frame rendered
    # with the result copied to the host (render.h:109-152). A first frame of >= 2^28
    # paths waits for the compile; a smaller one runs the generic flat kernel meanwhile.
    e2e = None
    if not a.no_e2e or a.e2e_only:
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        st, frame = step()
        host = (frame if frame is not None else part[: rows * W * 3]).cpu() if rank == 0 or world == 1 else None
        torch.cuda.synchronize()
        t_frame = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([t_build + t_scene + t_frame, float(st["rays"]), t_dev_init], dtype=torch.float64,
                              device=coll_dev)
            t_max = tt[[0, 2]].clone()
            dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
            dist.all_reduce(tt[1:2], op=dist.ReduceOp.SUM)
            e2e_s, e2e_rays, dev_init_s = float(t_max[0]), float(tt[1]), float(t_max[1])
        else:
            e2e_s, e2e_rays, dev_init_s = t_build + t_scene + t_frame, float(st["rays"]), t_dev_init
        del host
        e2e = {"value": e2e_rays / e2e_s / 1e6, "unit": "Mray/s", "seconds": e2e_s,
               "device_init_s": dev_init_s, "value_with_device_init": e2e_rays / (e2e_s + dev_init_s) / 1e6,
               "bvh_build_s": t_build, "set_scene_s": t_scene, "context_create_s": t_ctx, "frame_with_d2h_s": t_frame,
               "first_frame_kernel": ptamd._lib.pt_stats.PATHS.get(st["kernel_path"], "?")}
        log(f"[bench] end to end ({'warm code cache' if a.e2e_only else 'cold'}): {e2e_s:.3f} s, "
            f"first frame {t_frame:.3f} s on {e2e['first_frame_kernel']}")
        if a.e2e_only:
            os.write(JSON_FD, (json.dumps({"end_to_end": e2e}) + "\n").encode())
            r.close()
            return
        if world == 1 and scene_uses_rtc:
            e2e["warm"] = warm_e2e(a, rtc_dir)
    # steady state: the scene-specialised kernel is ready before the warm-up and timed steps
    r.prepare()
    for i in range(a.warmup):
        st, _ = step()
        log(f"[bench] warmup {i}: {st['rays']} rays, trace kernel {st['kernel_ms']:.1f} ms")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    rays = 0
    kms, launches = 0.0, 0
    render_s, gather_s = 0.0, 0.0
    kernel_name = "?"
    for i in range(a.steps):
        st, _ = step()
        rays += st["rays"]
        kms += st["kernel_ms"]
        launches += st["trace_launches"]
        render_s += st["render_s"]
        gather_s += st["gather_s"]
        kernel_name = ptamd._lib.pt_stats.PATHS.get(st["kernel_path"], "?")
        log(f"[bench] step {i}: {st['rays']} rays, trace kernel {st['kernel_ms']:.1f} ms over "
            f"{st['trace_launches']} launches, call {st['total_ms']:.1f} ms")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # what every rank saw: its device, its rows, its trace-kernel time and rays, its clock
    props = torch.cuda.get_device_properties(dev)
    mine = [float(rank), float(dev.index), float(getattr(props, "pci_bus_id", -1)),
            float(getattr(props, "pci_device_id", -1)), float(rows), kms, float(rays), float(launches), elapsed,
            render_s, gather_s]
    if world > 1:
        t = torch.tensor(mine, dtype=torch.float64, device=coll_dev)
        every = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(every, t)
        per_rank = [e.cpu().tolist() for e in every]
        elapsed = max(r[8] for r in per_rank)
        total_rays = sum(r[6] for r in per_rank)
    else:
        per_rank = [mine]
        total_rays = float(rays)
    # render_ms / gather_ms: host wall time per timed step of the rank's own rows and of the
    # gather to rank 0 (render + gather ~ ms_per_step; a scaling run separates the two)
    ranks = [{"rank": int(r[0]), "device": int(r[1]), "pci_bus_id": int(r[2]), "pci_device_id": int(r[3]),
              "rows": int(r[4]), "kernel_ms": r[5], "rays": int(r[6]), "trace_launches": int(r[7]),
              "wall_s": r[8], "render_ms": r[9] * 1e3 / a.steps, "gather_ms": r[10] * 1e3 / a.steps}
             for r in per_rank]
    world_info = {"world_size": dist.get_world_size() if world > 1 else 1,
                  "backend": dist.get_backend() if world > 1 else None, "launcher": launcher,
                  "process_groups": 1 if world > 1 else 0,
                  "rccl_version": ".".join(map(str, torch.cuda.nccl.version())) if world > 1 and backend == "nccl"
                  else None,
                  "distinct_devices": len({(r["pci_bus_id"], r["pci_device_id"], r["device"]) for r in ranks}),
                  "ranks": ranks}

    # ---- rooflines of the dominant kernel (the trace kernel), per launch
    workload = f"{scene.name}_{W}x{H}_spp{a.spp}_depth{a.depth}"
    avg_launch_s = (kms / 1e3) / max(launches, 1)
    rays_per_launch = rays / max(launches, 1)
    b_ray = B_RAY.get((a.scene, a.depth), B_RAY[("cornell", 5)])
    pm, pm_src = load_pmc(f"{scene.name}_{W}x{H}_depth{a.depth}")
    valu = None
    if pm and avg_launch_s > 0 and pm.get("valu_main_slots_per_ray"):
        ach = pm["valu_main_slots_per_ray"] * rays_per_launch / avg_launch_s / 1e9
        valu = {"bound": "valu", "achieved": ach, "peak": VALU_PEAK_G, "unit": "G VALU main-port slots/s",
                "frac": ach / VALU_PEAK_G, "valu_main_slots_per_ray": pm["valu_main_slots_per_ray"],
                "valu_second_port_slots_per_ray": pm.get("valu_second_port_slots_per_ray"),
                "valu_insts_per_ray": pm["valu_insts_per_ray"], "valu_lane_utilisation": pm.get("valu_lane_utilisation")}
    # the binding roofline at the nominal 2.4 GHz the peak assumes, at the clock the keyed PMC
    # pass measured (GRBM_GUI_ACTIVE / time), and the headroom in useful lanes: frac x the
    # fraction of issued VALU lanes that were active (SQ_THREAD_CYCLES_VALU / 64 per instruction)
    clk = pm.get("gpu_clock_ghz_grbm") if pm else None
    lanes = pm.get("valu_lane_utilisation") if pm else None
    roofline = {"bound": "valu", "achieved": valu["achieved"] if valu else None, "peak": VALU_PEAK_G,
                "unit": "G VALU main-port slots/s", "frac": valu["frac"] if valu else None,
                "clock_ghz_nominal": 2.4, "clock_ghz_measured": clk,
                "frac_at_measured_clock": valu["frac"] * 2.4 / clk if valu and clk else None,
                "useful_lane_frac": valu["frac"] * lanes if valu and lanes else None,
                "traffic": pm["hbm_bytes_per_ray"] * rays_per_launch if pm else None,
                "kernel": kernel_name, "avg_launch_ms": avg_launch_s * 1e3, "rays_per_launch": rays_per_launch,
                "valu_main_slots_per_ray": pm.get("valu_main_slots_per_ray") if pm else None,
                "valu_insts_per_ray": pm["valu_insts_per_ray"] if pm else None,
                "valu_lane_utilisation": pm.get("valu_lane_utilisation") if pm else None,
                "pmc_key": kernel_key(), "pmc_source": pm_src}
    # the guide's model (MI355X_MICROARCH.md: v_fma_f32 wave64 at 2 cycles with several waves
    # per SIMD, 1,228.8 G instructions/s, every VALU instruction one slot) beside the calibrated
    # one above (4 cycles, second-port forms free; DESIGN.md §5, profiles/r05_valu_peak)
    if pm and avg_launch_s > 0:
        ach2 = pm["valu_insts_per_ray"] * rays_per_launch / avg_launch_s / 1e9
        roofline["model_2cyc"] = {"achieved": ach2, "peak": 2 * VALU_PEAK_G, "unit": "G VALU instructions/s",
                                  "frac": ach2 / (2 * VALU_PEAK_G)}
        roofline["valu_insts_issue_frac_2cyc_model"] = ach2 / (2 * VALU_PEAK_G)
    alg = rays_per_launch * b_ray / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    hbm_alg = {"bytes_per_ray": b_ray, "achieved": alg, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "ratio_vs_peak": alg / HBM_PEAK_GBS, "applicable": False,
               "note": "reference-layout bytes (SURVEY.md §8(d)); the scene is LDS/constant/L2-resident, "
                       "so this is not HBM traffic and the ratio is not a roofline fraction"}
    hbm_meas = None
    if pm and avg_launch_s > 0:
        gbs = pm["hbm_bytes_per_ray"] * rays_per_launch / avg_launch_s / 1e9
        hbm_meas = {"bytes_per_ray": pm["hbm_bytes_per_ray"], "achieved": gbs, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS}

    value = total_rays / elapsed / 1e6
    out = {
        "metric": "Mray/s (all bounces) + achieved HBM GB/s, Cornell 1024² 10k spp depth-5",
        "value": value,
        "unit": "Mray/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "strong",
        # README.md:23-29 quotes 112 s for this frame on the reference's GL
        # path; at the measured 3.534 segments per path that is ~331 Mray/s.
        "vs_baseline": value / README_MRAYS if (a.scene, a.res, a.spp, a.depth) == ("cornell", 1024, 10000, 5)
        and not a.part
        else None,
        "dtype": "f32",
        "data": f"synthetic ({scene.name} scene generated in-process)",
        "config": {"workload": workload, "scene": scene.name, "tris": len(scene.tris),
                   "res": [W, H], "spp": a.spp, "depth": a.depth, "seed": 1,
                   "parallelism": (f"rows dealt in {a.band}-row bands over {world} ranks, "
                                   f"{'RCCL' if backend == 'nccl' else backend} gather of the frame to rank 0")
                   if world > 1 else f"1 GPU, part {a.part} of the row partition only" if a.part
                   else "1 GPU, whole frame"},
        "roofline": roofline,
        "valu_issue": valu,
        "hbm_algorithmic": hbm_alg,
        "hbm_measured": hbm_meas,
        "rays_per_step": total_rays / a.steps,
        "kernel_mrays": rays / (kms / 1e3) / 1e6 if kms > 0 else None,
        "world": world_info,
    }

    if e2e is not None:
        e2e["kernel_only_mrays"] = out["kernel_mrays"]
        out["end_to_end"] = e2e
        if a.scene == "sphere":
            try:
                with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
                    g = json.load(f)
                out["end_to_end"]["reference_bvh_build_s"] = g["bvh_hash"]["sphere223_in_cornell"]["ref_build_s"]
            except (OSError, KeyError):
                pass
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        log("[bench] cpu baseline (reference, 1 core) ...")
        out["cpu_baseline"] = cpu_baseline(a, scene, bvh, r, cam)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        line = json.dumps(out) + "\n"
        if result_path:
            with open(result_path, "w") as f:
                f.write(line)
        else:
            os.write(JSON_FD, line.encode())
    r.close()
    if world > 1:
        dist.destroy_process_group()


# stdout carries exactly one line, the JSON result: everything else written to file
# descriptor 1 while the bench runs (Python prints, and C/C++ libraries such as gloo's
# "connected to N peer ranks" notice) is sent to stderr.
JSON_FD = 1

if __name__ == "__main__":
    sys.stdout.flush()
    JSON_FD = os.dup(1)
    os.dup2(2, 1)
    main()
