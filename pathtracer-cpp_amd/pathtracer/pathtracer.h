// pathtracer.h — drop-in replacement for the reference's umbrella header
// (Blackgaurd/pathtracer-cpp pathtracer/pathtracer.h:1-10). Programs written
// against the reference compile unchanged with
//   -I<repo>/pathtracer-cpp_amd -I<repo>/include  ... -L<repo>/pathtracer-cpp_amd/lib -lpt_hip
// and their render_cpu()/render_gpu() calls run the gfx950 trace kernel.
#pragma once

static_assert(__cplusplus >= 201703L, "C++17 required");

#include "pt_camera.hpp"
#include "pt_image.hpp"
#include "pt_linalg.hpp"
#include "pt_render.hpp"
#include "pt_scene.hpp"
