// pt_image.hpp — Image of the drop-in API (reference: pathtracer/image.h).
// pixels[h][w], h = 0 the bottom row; PNG/PPM writers flip vertically and
// quantise with (uchar)(clamp(x, 0, 1) * 255) as the reference does. PNG bytes
// come from libpt_hip.so's zlib writer (the reference uses fpng; the decoded
// pixels are identical).
#pragma once

#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "pt_hip.h"
#include "pt_linalg.hpp"

struct Image {
    ivec2 res;
    std::vector<std::vector<vec3>> pixels;

    Image() = default;
    Image(const ivec2& r) : res(r), pixels(r.y, std::vector<vec3>(r.x, vec3(0.0f))) {}

    void set_pixel(int w, int h, const vec3& c) { at(w, h) = c; }
    vec3 get_pixel(int w, int h) const { return const_cast<Image*>(this)->at(w, h); }
    vec3& get_pixel(int w, int h) { return at(w, h); }
    void operator+=(const Image& o) {
        if (res != o.res) throw std::invalid_argument("image resolution mismatch");
        for (int h = 0; h < res.y; h++)
            for (int w = 0; w < res.x; w++) pixels[h][w] += o.pixels[h][w];
    }
    void operator/=(float s) {
        for (auto& row : pixels)
            for (vec3& p : row) p /= s;
    }
    void gamma_correct(float gamma) {
        for (auto& row : pixels)
            for (vec3& p : row) p = pow(p, 1 / gamma);
    }
    std::vector<unsigned char> rgb8() const {  // top row first
        std::vector<unsigned char> d((size_t)res.x * res.y * 3);
        for (int h = 0; h < res.y; h++)
            for (int w = 0; w < res.x; w++) {
                const vec3& p = pixels[res.y - h - 1][w];
                unsigned char* o = &d[((size_t)h * res.x + w) * 3];
                o[0] = static_cast<unsigned char>(clamp(p.x, 0, 1) * 255);
                o[1] = static_cast<unsigned char>(clamp(p.y, 0, 1) * 255);
                o[2] = static_cast<unsigned char>(clamp(p.z, 0, 1) * 255);
            }
        return d;
    }
    void save_png(std::string filename) {
        const std::vector<unsigned char> d = rgb8();
        if (pt_write_png(filename.c_str(), d.data(), res.x, res.y) != PT_OK)
            std::cerr << "Failed to write image to file: " << filename << '\n';
    }
    void save_ppm(std::string filename) {
        const std::vector<unsigned char> d = rgb8();
        std::ofstream out(filename, std::ios::binary);
        out << "P6\n" << res.x << " " << res.y << "\n255\n";
        out.write(reinterpret_cast<const char*>(d.data()), (std::streamsize)d.size());
    }

   private:
    vec3& at(int w, int h) {
        if (w < 0 || w >= res.x || h < 0 || h >= res.y) throw std::out_of_range("pixel out of range");
        return pixels[h][w];
    }
};
