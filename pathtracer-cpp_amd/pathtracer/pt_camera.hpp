// pt_camera.hpp — Camera of the drop-in API (reference: pathtracer/camera.h).
// The ctor's derived parameters (v_res, cell_size, transform) come from
// libpt_hip.so's pt_camera_init, the same arithmetic the reference performs;
// get_ray/rotate/move keep the reference's member semantics.
#pragma once

#include <array>
#include <cstring>
#include <iostream>

#include "pt_hip.h"
#include "pt_linalg.hpp"
#include "pt_scene.hpp"

struct Camera {
    enum Direction { FORWARD, BACKWARD, LEFT, RIGHT, UP, DOWN };

    ivec2 res;
    vec2 v_res;
    float fov, distance, cell_size;
    vec3 pos;
    vec3 forward, up, right;
    vec3 world_up;
    std::array<float, 16> transform;

    Camera() = default;
    Camera(const vec3& pos_, const vec3& forward_, const vec3& up_, const ivec2& res_, float fov_, float distance_) {
        pos = pos_;
        forward = forward_.normalize();
        right = forward_.cross(up_).normalize();
        up = up_.normalize();
        world_up = up;
        pt_camera c;
        const float p[3] = {pos_.x, pos_.y, pos_.z}, f[3] = {forward_.x, forward_.y, forward_.z},
                    u[3] = {up_.x, up_.y, up_.z};
        if (pt_camera_init(p, f, u, res_.x, res_.y, fov_, distance_, &c) != PT_OK) {
            std::cerr << "Up vector is too close to forward vector" << '\n';
            std::cerr << "forward: " << forward << ", up: " << up << '\n';
            return;
        }
        res = res_;
        fov = fov_;
        distance = distance_;
        v_res = vec2(c.v_res[0], c.v_res[1]);
        cell_size = c.cell_size;
        transform.fill(0.0f);
        for (int i = 0; i < 4; i++) transform[i * 4 + i] = 1;
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 3; k++) transform[r * 4 + k] = c.transform[r * 3 + k];
        set_row(3, pos);
    }

    // camera.h:63-73 with the global rng; the y jitter is drawn first (g++ order).
    void get_ray(int w, int h, vec3& ray_o, vec3& ray_d) const {
        const float jy = rng.rand01();
        const float jx = rng.rand01();
        const vec3 c((w + jx) * cell_size - v_res.x / 2, (h + jy) * cell_size - v_res.y / 2, -distance);
        ray_d = vec3(c.dot(vec3(transform[0], transform[4], transform[8])),
                     c.dot(vec3(transform[1], transform[5], transform[9])),
                     c.dot(vec3(transform[2], transform[6], transform[10])))
                    .normalize();
        ray_o = pos;
    }

    // The C ABI view of this camera.
    pt_camera to_c() const {
        pt_camera c;
        std::memset(&c, 0, sizeof(c));
        c.pos[0] = pos.x; c.pos[1] = pos.y; c.pos[2] = pos.z;
        c.res[0] = res.x; c.res[1] = res.y;
        c.v_res[0] = v_res.x; c.v_res[1] = v_res.y;
        c.cell_size = cell_size;
        c.distance = distance;
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 3; k++) c.transform[r * 3 + k] = transform[r * 4 + k];
        return c;
    }

    void rotate(Direction dir, float angle) {
        switch (dir) {
            case LEFT:
            case RIGHT: {
                const float s = dir == LEFT ? -std::sin(angle) : std::sin(angle);
                forward = (forward * std::cos(angle) + right * s).normalize();
                right = forward.cross(world_up).normalize();
                up = right.cross(forward).normalize();
                break;
            }
            case UP:
            case DOWN: {
                const float s = dir == DOWN ? -std::sin(angle) : std::sin(angle);
                forward = (forward * std::cos(angle) + up * s).normalize();
                up = right.cross(forward).normalize();
                break;
            }
            default: break;
        }
        set_row(0, right);
        set_row(1, up);
        set_row(2, -forward);
    }
    void move(Direction dir, float amount) {
        const vec3 level_forward = world_up.cross(right).normalize();
        switch (dir) {
            case UP: pos += world_up * amount; break;
            case DOWN: pos -= world_up * amount; break;
            case FORWARD: pos += level_forward * amount; break;
            case BACKWARD: pos -= level_forward * amount; break;
            case LEFT: pos -= right * amount; break;
            case RIGHT: pos += right * amount; break;
        }
        set_row(3, pos);
    }

   private:
    void set_row(int r, const vec3& v) {
        transform[r * 4] = v.x;
        transform[r * 4 + 1] = v.y;
        transform[r * 4 + 2] = v.z;
    }
};
