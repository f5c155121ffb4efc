// Internal helpers of the host surface (not part of the ABI).
//
// The reference's host code does its vector math with glm 0.9.9.7 in plain
// IEEE single precision (x86-64 SSE, no contraction).  V3 below reproduces the
// operation order of the glm functions the host path uses:
//   glm::min/max   (y < x) ? y : x               (glm/detail/func_common.inl)
//   glm::dot       (x*x' + y*y') + z*z'          (func_geometric.inl)
//   glm::cross     (y*z' - y'*z, z*x' - z'*x, x*y' - x'*y)
//   glm::normalize v * (1 / sqrt(dot(v, v)))     (func_geometric.inl:82-89)
// This file is compiled with -ffp-contract=off.
#pragma once

#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/rt2.h"

namespace rt2h {

struct V3 {
    float x = 0.0f, y = 0.0f, z = 0.0f;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit V3(float s) : x(s), y(s), z(s) {}
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(V3 a, V3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator-(V3 a) { return V3(-a.x, -a.y, -a.z); }
inline V3 operator*(V3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
inline V3 operator*(float s, V3 a) { return V3(s * a.x, s * a.y, s * a.z); }
inline V3 operator/(V3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
inline float gmin(float x, float y) { return (y < x) ? y : x; }
inline float gmax(float x, float y) { return (x < y) ? y : x; }
inline V3 vmin(V3 a, V3 b) { return V3(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
inline V3 vmax(V3 a, V3 b) { return V3(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }
inline float gdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 gcross(V3 x, V3 y) {
    return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
inline V3 gnormalize(V3 v) { return v * (1.0f / std::sqrt(gdot(v, v))); }

inline V3 xyz(const rt2_vec4& v) { return V3(v.x, v.y, v.z); }
inline rt2_vec4 vec4(V3 v, float w = 0.0f) { return rt2_vec4{v.x, v.y, v.z, w}; }

// BVHTriangle, mesh.h:141-154.
struct BvhTri {
    V3 min, max, center;
    BvhTri() = default;
    BvhTri(V3 a, V3 b, V3 c) {
        min = vmin(vmin(a, b), c);
        max = vmax(vmax(a, b), c);
        center = ((a + b) + c) / 3.0f;
    }
};

// BoundingBox, BVH.h:11-52 — including size() returning the x-extent in all
// three components (BVH.h:30-33), which the reference's builders and SAH use.
struct Box {
    V3 min = V3(1e30f);
    V3 max = V3(-1e30f);
    V3 size() const { return V3(max[0] - min[0], max[0] - min[0], max[0] - min[0]); }
    void grow(const BvhTri& t) {
        min = vmin(min, t.min);
        max = vmax(max, t.max);
    }
    void expand() {
        min = min - V3(1e-4f);
        max = max + V3(1e-4f);
    }
};

// A decoded 8-bit image (stb_image's stbi_load result layout: rows of w*n
// bytes, no padding, row 0 = first row in memory).
struct Image {
    int w = 0, h = 0, n = 0;
    std::vector<uint8_t> px;
};
// stbi_load(path, ..., 0) after stbi_set_flip_vertically_on_load(flip)
// (image.cpp); throws std::runtime_error on unsupported/corrupt files.
Image load_image(const std::string& path, bool flip);

struct SceneData {
    std::vector<rt2_triangle> tris;
    std::vector<BvhTri> btris;
    std::vector<rt2_material> mats;
    std::vector<std::string> tex_names;
    std::vector<Image> textures;  // decoded, flipped on load (textureClass.cpp:55-68)
    std::vector<rt2_node> nodes;

    void push(const rt2_triangle& t) {
        tris.push_back(t);
        btris.emplace_back(xyz(t.a), xyz(t.b), xyz(t.c));
    }
    void push_tri(int mtl, V3 a, V3 b, V3 c) {
        rt2_triangle t{};
        t.a = vec4(a);
        t.b = vec4(b);
        t.c = vec4(c);
        t.materialIndex = mtl;
        push(t);
    }
    Box bounds() const {
        Box b;
        for (const BvhTri& t : btris) b.grow(t);
        return b;
    }
};

// Error plumbing: C++ exceptions stop at the ABI.
void set_error(const std::string& msg);
template <class F>
int guard(F&& f) {
    try {
        return f();
    } catch (const std::exception& e) {
        set_error(e.what());
        return -1;
    } catch (...) {
        set_error("unknown error");
        return -1;
    }
}

}  // namespace rt2h

struct rt2_scene_data : rt2h::SceneData {};
