#!/usr/bin/env python3
"""Offline ISA of the hipRTC scene-specialised flat kernel (no GPU needed).

Generates the kernel source for a scene through pt_rtc_check (the same generator
pt_ctx_set_scene uses), compiles it with hipcc for gfx950 with the hipRTC numerics
flags, and prints the kernel's register use and the VALU / SALU / LDS instruction
count of every basic block (the largest first), so a source change can be judged
before a GPU run.
usage: python scripts/rtc_isa.py [cornell|mcornell] [-D NAME=VALUE ...] [--out DIR]
"""
import argparse
import ctypes as C
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))

# pt_kernel.hip: rtc_compile's flags (bit parity depends on the numerics ones)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero", "-fno-slp-vectorize",
         "-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-use-amdgpu-trackers"]


def source(scene_name):
    import ptamd as pt
    from ptamd import scenes
    sc = scenes.cornell((8, 8)) if scene_name == "cornell" else scenes.modified_cornell(0.3, (8, 8))
    ref = pt._SceneRef(pt.BVH.from_scene(sc))
    buf = C.create_string_buffer(1 << 20)
    if pt.lib().pt_rtc_check(C.byref(ref.s), buf, len(buf)) <= 0:
        raise SystemExit(pt.lib().pt_last_error().decode())
    src = buf.value.decode()
    # hipRTC-only preamble -> the offline compiler's headers
    src = "\n".join(l for l in src.split("\n") if "__hip_internal" not in l)
    src = src.replace("#if !defined(__HIP_DEVICE_COMPILE__)\n#error", "#if 0\n#error")
    return "#include <hip/hip_runtime.h>\n#include <stdint.h>\n" + src


def blocks(asm):
    out, cur = [], None
    body = asm[asm.index("pt_trace_flat_rtc:"):]
    body = body[:body.index("s_endpgm")]
    for line in body.split("\n"):
        m = re.match(r"^(\.LBB\d+_\d+):|^; %bb\.(\d+):", line)
        if m:
            cur = {"name": m.group(1) or "bb." + m.group(2), "v": 0, "s": 0, "ds": 0, "mem": 0, "lane": 0}
            out.append(cur)
            continue
        s = line.strip()
        if cur is None or not s or s[0] in ";.":
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            cur["v"] += 1
            cur["lane"] += "readlane" in op or "writelane" in op
        elif op.startswith("s_"):
            cur["s"] += 1
        elif op.startswith("ds_"):
            cur["ds"] += 1
        elif op.startswith(("global_", "buffer_", "scratch_", "flat_")):
            cur["mem"] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene", nargs="?", default="cornell", choices=["cornell", "mcornell"])
    ap.add_argument("-D", action="append", default=[], help="macro for the generated source (PT_RTC_DEFINES)")
    ap.add_argument("--out", default="/tmp/rtc_isa")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    src = "".join(f"#define {d.replace('=', ' ', 1)}\n" for d in a.D) + source(a.scene)
    hip = os.path.join(a.out, f"{a.scene}.hip")
    asm_path = os.path.join(a.out, f"{a.scene}.s")
    with open(hip, "w") as f:
        f.write(src)
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "pathtracer-cpp_amd", "csrc")]
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *inc, "-S", "--offload-device-only", hip, "-o", asm_path],
                   check=True, stderr=subprocess.DEVNULL)
    asm = open(asm_path).read()
    for key in ("NumVgprs", "NumSgprs", "ScratchSize", "Occupancy"):
        m = re.search(rf"; {key}: (\d+)", asm)
        print(f"{key}: {m.group(1) if m else '?'}")
    bl = blocks(asm)
    print(f"blocks {len(bl)}, VALU {sum(b['v'] for b in bl)}, SGPR-spill lane ops {sum(b['lane'] for b in bl)}, "
          f"scratch ops {asm.count('scratch_')}")
    for b in sorted(bl, key=lambda b: -b["v"])[: a.top]:
        print(f"  {b['name']:12s} valu {b['v']:4d}  salu {b['s']:3d}  lds {b['ds']:2d}  vmem {b['mem']:2d}  "
              f"spill-lane {b['lane']:2d}")
    print(f"source {hip}, ISA {asm_path}")


if __name__ == "__main__":
    main()
