#!/usr/bin/env bash
# Build oracle/_ref/pt_ref — the UNMODIFIED reference CPU path (test infrastructure).
#
# Recipe: compile the reference's own sources where they
# lie under $PT_REFERENCE (default /root/reference) with the reference's copts
# (-std=c++17 -O3, examples/BUILD.bazel:6-9; fpng with -DFPNG_NO_SSE -w,
# pathtracer/BUILD.bazel:3-12). render.h cannot be included whole (it pulls in
# SFML and the GL shader, render.h:3,14), so its CPU part — lines 16-108:
# SHIFT_BIAS, Timer, trace, render_cpu, ceildiv — is extracted verbatim into a
# temporary directory that is deleted after the compile. No reference source is
# written into the repository; only the binary lands in oracle/_ref/.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
REF="${PT_REFERENCE:-/root/reference}"
OUT="$REPO/oracle/_ref"
CXX="${CXX:-g++}"

if [ ! -f "$REF/pathtracer/render.h" ]; then
    echo "build_ref.sh: reference not found at $REF (skipping; prebuilt $OUT/pt_ref is used if present)" >&2
    exit 0
fi
mkdir -p "$OUT"
TMP="$(mktemp -d)"
trap 'rm -rf "$TMP"' EXIT

# Guard the extraction window against a changed reference.
first="$(sed -n '16p' "$REF/pathtracer/render.h")"
last="$(sed -n '106,108p' "$REF/pathtracer/render.h" | tr -d '\n')"
if [ "$first" != "#define SHIFT_BIAS 1e-4" ] || [ "$last" != "int ceildiv(int a, int b) {    return (a + b - 1) / b;}" ]; then
    echo "build_ref.sh: render.h layout changed; refusing to extract" >&2
    exit 1
fi
sed -n '16,108p' "$REF/pathtracer/render.h" > "$TMP/render_cpu_part.h"

"$CXX" -std=c++17 -O3 -DFPNG_NO_SSE -w -c "$REF/pathtracer/fpng.cc" -o "$TMP/fpng.o"
"$CXX" -std=c++17 -O3 -w -c "$REF/pathtracer/tiny_obj_loader.cc" -o "$TMP/tiny_obj_loader.o"
"$CXX" -std=c++17 -O3 -I"$REF" -I"$TMP" -I"$REPO/include" \
    "$HERE/pt_ref_harness.cc" "$TMP/fpng.o" "$TMP/tiny_obj_loader.o" -o "$OUT/pt_ref"
echo "built $OUT/pt_ref"

# The reference's own example programs, compiled UNCHANGED against the drop-in headers
# (pathtracer-cpp_amd/pathtracer/pathtracer.h) and linked to libpt_hip.so: evidence that
# the boundary is a drop-in. Outputs only into oracle/_ref/.
PKG="$REPO/pathtracer-cpp_amd"
if [ -f "$PKG/lib/libpt_hip.so" ]; then
    for src in examples/cornell_box.cc examples/modified_cornell.cc tests/test_render.cc; do
        name="dropin_$(basename "$src" .cc)"
        "$CXX" -std=c++17 -O3 -I"$PKG" -I"$REPO/include" "$REF/$src" -L"$PKG/lib" -lpt_hip \
            -Wl,-rpath,'$ORIGIN/../../pathtracer-cpp_amd/lib' -o "$OUT/$name"
    done
    echo "built $OUT/dropin_{cornell_box,modified_cornell,test_render}"
fi
