// Scene assembly of the host surface: material helpers (mesh.h:47-102), the
// Cornell-box builders of RayTracing/src/rayTracing.cpp, the BVH build that
// fixes the triangle order (BVH.h:117-221), and scene-data accessors.
//
// Deliberate deviation (SURVEY.md §7 "Reference UB"): addCornellBox builds the
// light's BVH triangles with the 12-row wall index table, reading
// lightCorners[4], [5] of a 4-element vector (rayTracing.cpp:537).  Here every
// BVH triangle is built from its own render triangle's vertices, i.e. with the
// light-corner table of :512-518.  Everything else — including the x-extent
// BoundingBox::size() (BVH.h:30-33) that sizes the boxes — is as written.
#include <cstring>

#include "host_internal.h"

using namespace rt2h;

namespace rt2h {
thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace rt2h

extern "C" const char* rt2_last_error(void) { return rt2h::g_last_error.c_str(); }
extern "C" int rt2_abi_version(void) { return RT2_ABI_VERSION; }

/* ---- materials, mesh.h:26-103 ------------------------------------------ */
extern "C" void rt2_material_default(rt2_material* m) {
    std::memset(m, 0, sizeof(*m));
    m->color = rt2_vec4{1.0f, 1.0f, 1.0f, 0.0f};
    m->textureIndex = -1;
    m->materialType = RT2_DIFFUSE;
}
extern "C" void rt2_material_make_diffuse(rt2_material* m, float r, float g, float b) {
    m->materialType = RT2_DIFFUSE;
    m->color = rt2_vec4{r, g, b, 0.0f};
}
extern "C" void rt2_material_make_light(rt2_material* m, float r, float g, float b, float strength) {
    m->materialType = RT2_LIGHT;
    m->emissionColor = rt2_vec4{r, g, b, 0.0f};
    m->emissionStrength = strength;
}
extern "C" void rt2_material_make_specular(rt2_material* m, float r, float g, float b, float sr, float sg, float sb,
                                           float smooth, float prob) {
    m->materialType = RT2_SPECULAR;
    m->color = rt2_vec4{r, g, b, 0.0f};
    m->specularColor = rt2_vec4{sr, sg, sb, 0.0f};
    m->smoothness = smooth;
    m->specularProbability = prob;
}
extern "C" void rt2_material_make_checker(rt2_material* m, float scale) {
    m->materialType = RT2_CHECKER;
    m->checkerScale = scale;
}
extern "C" void rt2_material_make_glass(rt2_material* m, float r, float g, float b, float ior) {
    m->materialType = RT2_GLASS;
    m->color = rt2_vec4{r, g, b, 0.0f};
    m->refractiveIndex = ior;
}

/* ---- scene data ----------------------------------------------------------- */
extern "C" rt2_scene_data* rt2_sd_create(void) {
    try {
        return new rt2_scene_data();
    } catch (...) {
        set_error("out of memory");
        return nullptr;
    }
}
extern "C" void rt2_sd_destroy(rt2_scene_data* sd) { delete sd; }

extern "C" int32_t rt2_sd_add_material(rt2_scene_data* sd, const rt2_material* m) {
    if (!sd || !m) {
        set_error("null argument");
        return -1;
    }
    sd->mats.push_back(*m);
    return (int32_t)sd->mats.size() - 1;
}

extern "C" int rt2_sd_add_triangle(rt2_scene_data* sd, const float a[3], const float b[3], const float c[3],
                                   int32_t mtl) {
    if (!sd || !a || !b || !c) {
        set_error("null argument");
        return -1;
    }
    sd->push_tri(mtl, V3(a[0], a[1], a[2]), V3(b[0], b[1], b[2]), V3(c[0], c[1], c[2]));
    return 0;
}

extern "C" int rt2_sd_add_triangles(rt2_scene_data* sd, const rt2_triangle* tris, int32_t n) {
    if (!sd || (n > 0 && !tris) || n < 0) {
        set_error("bad argument");
        return -1;
    }
    for (int32_t i = 0; i < n; i++) sd->push(tris[i]);
    return 0;
}

extern "C" int32_t rt2_sd_num_triangles(const rt2_scene_data* sd) { return sd ? (int32_t)sd->tris.size() : 0; }
extern "C" int32_t rt2_sd_num_materials(const rt2_scene_data* sd) { return sd ? (int32_t)sd->mats.size() : 0; }
extern "C" int32_t rt2_sd_num_nodes(const rt2_scene_data* sd) { return sd ? (int32_t)sd->nodes.size() : 0; }
extern "C" int rt2_sd_texture(const rt2_scene_data* sd, int32_t i, rt2_image* out) {
    if (!sd || !out || i < 0 || i >= (int32_t)sd->textures.size()) {
        rt2h::set_error("rt2_sd_texture: bad argument");
        return -1;
    }
    const rt2h::Image& im = sd->textures[i];
    out->width = im.w;
    out->height = im.h;
    out->channels = im.n;
    out->pixels = const_cast<uint8_t*>(im.px.data());
    return 0;
}

extern "C" int32_t rt2_sd_num_textures(const rt2_scene_data* sd) { return sd ? (int32_t)sd->tex_names.size() : 0; }
extern "C" const rt2_triangle* rt2_sd_triangles(const rt2_scene_data* sd) { return sd ? sd->tris.data() : nullptr; }
extern "C" const rt2_material* rt2_sd_materials(const rt2_scene_data* sd) { return sd ? sd->mats.data() : nullptr; }
extern "C" const rt2_node* rt2_sd_nodes(const rt2_scene_data* sd) { return sd ? sd->nodes.data() : nullptr; }
extern "C" const char* rt2_sd_texture_name(const rt2_scene_data* sd, int32_t i) {
    if (!sd || i < 0 || i >= (int32_t)sd->tex_names.size()) return nullptr;
    return sd->tex_names[i].c_str();
}
extern "C" int rt2_sd_bvh_triangles(const rt2_scene_data* sd, float* out9) {
    if (!sd || !out9) return -1;
    for (size_t i = 0; i < sd->btris.size(); i++) {
        const BvhTri& t = sd->btris[i];
        float v[9] = {t.min.x, t.min.y, t.min.z, t.max.x, t.max.y, t.max.z, t.center.x, t.center.y, t.center.z};
        std::memcpy(out9 + 9 * i, v, sizeof(v));
    }
    return 0;
}

/* ---- builders, rayTracing.cpp --------------------------------------------- */
namespace {

struct Padded {
    float minX, maxX, minY, maxY, minZ, maxZ;
    V3 sceneSize;
};

// The padded scene box shared by addCornellBox / addMirrorCornellBox /
// addSideLitCornellBox (rayTracing.cpp:455-465 and copies).
Padded padded_box(const SceneData& sd, float pad) {
    Box b = sd.bounds();
    V3 s = b.size();
    Padded p;
    p.sceneSize = s;
    p.minX = b.min.x - s.x * pad;
    p.maxX = b.max.x + s.x * pad;
    p.minY = b.min.y - s.y * pad * 0.1f;
    p.maxY = b.max.y + s.y * pad;
    p.minZ = b.min.z - s.z * pad;
    p.maxZ = b.max.z + s.z * pad;
    return p;
}

void box_corners(const Padded& p, V3 c[8]) {
    c[0] = V3(p.minX, p.minY, p.maxZ);
    c[1] = V3(p.maxX, p.minY, p.maxZ);
    c[2] = V3(p.minX, p.maxY, p.maxZ);
    c[3] = V3(p.maxX, p.maxY, p.maxZ);
    c[4] = V3(p.minX, p.minY, p.minZ);
    c[5] = V3(p.maxX, p.minY, p.minZ);
    c[6] = V3(p.minX, p.maxY, p.minZ);
    c[7] = V3(p.maxX, p.maxY, p.minZ);
}

// Wall winding of the mirror / side-lit boxes (rayTracing.cpp:611-625).
const int kWalls[12][3] = {{0, 3, 1}, {0, 2, 3}, {0, 5, 4}, {0, 1, 5}, {0, 6, 2}, {0, 4, 6},
                           {1, 7, 5}, {1, 3, 7}, {2, 7, 3}, {2, 6, 7}, {4, 7, 6}, {4, 5, 7}};

// 4x4 column-major matrix with glm's operation order (glm/ext/matrix_transform.inl:18-46,
// glm/detail/type_mat4x4.inl:536-648).
struct M4 {
    float m[4][4];  // m[col][row]
};
M4 identity() {
    M4 r{};
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0f;
    return r;
}
// column * scalar + column * scalar + ... left to right
void col_lin3(const M4& a, float s0, float s1, float s2, float out[4]) {
    for (int r = 0; r < 4; r++) out[r] = a.m[0][r] * s0 + a.m[1][r] * s1 + a.m[2][r] * s2;
}
M4 rotate(const M4& m, float angle, V3 v) {
    const float c = std::cos(angle);
    const float s = std::sin(angle);
    V3 axis = gnormalize(v);
    V3 temp = (1.0f - c) * axis;
    float R[3][3];
    R[0][0] = c + temp[0] * axis[0];
    R[0][1] = temp[0] * axis[1] + s * axis[2];
    R[0][2] = temp[0] * axis[2] - s * axis[1];
    R[1][0] = temp[1] * axis[0] - s * axis[2];
    R[1][1] = c + temp[1] * axis[1];
    R[1][2] = temp[1] * axis[2] + s * axis[0];
    R[2][0] = temp[2] * axis[0] + s * axis[1];
    R[2][1] = temp[2] * axis[1] - s * axis[0];
    R[2][2] = c + temp[2] * axis[2];
    M4 out;
    for (int k = 0; k < 3; k++) col_lin3(m, R[k][0], R[k][1], R[k][2], out.m[k]);
    for (int r = 0; r < 4; r++) out.m[3][r] = m.m[3][r];
    return out;
}
M4 mat_mul(const M4& a, const M4& b) {
    M4 out;
    for (int k = 0; k < 4; k++)
        for (int r = 0; r < 4; r++)
            out.m[k][r] = a.m[0][r] * b.m[k][0] + a.m[1][r] * b.m[k][1] + a.m[2][r] * b.m[k][2] + a.m[3][r] * b.m[k][3];
    return out;
}
// mat4 * vec4 (type_mat4x4.inl:561-575): (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
void mat_vec(const M4& a, const float v[4], float out[4]) {
    for (int r = 0; r < 4; r++) {
        float add0 = a.m[0][r] * v[0] + a.m[1][r] * v[1];
        float add1 = a.m[2][r] * v[2] + a.m[3][r] * v[3];
        out[r] = add0 + add1;
    }
}

void add_cube(SceneData& sd, V3 center, V3 size, V3 rotation, int mtl) {
    M4 I = identity();
    M4 rx = rotate(I, rotation.x, V3(1, 0, 0));
    M4 ry = rotate(I, rotation.y, V3(0, 1, 0));
    M4 rz = rotate(I, rotation.z, V3(0, 0, 1));
    M4 rot = mat_mul(mat_mul(rz, ry), rx);
    V3 h = size * 0.5f;
    V3 v[8] = {V3(-h.x, -h.y, +h.z), V3(+h.x, -h.y, +h.z), V3(-h.x, +h.y, +h.z), V3(+h.x, +h.y, +h.z),
               V3(-h.x, -h.y, -h.z), V3(+h.x, -h.y, -h.z), V3(-h.x, +h.y, -h.z), V3(+h.x, +h.y, -h.z)};
    for (V3& p : v) {
        float in[4] = {p.x, p.y, p.z, 1.0f}, o[4];
        mat_vec(rot, in, o);
        p = V3(o[0], o[1], o[2]) + center;
    }
    static const int f[12][3] = {{0, 1, 3}, {0, 3, 2}, {1, 5, 7}, {1, 7, 3}, {5, 4, 6}, {5, 6, 7},
                                 {4, 0, 2}, {4, 2, 6}, {2, 3, 7}, {2, 7, 6}, {4, 5, 1}, {4, 1, 0}};
    for (int i = 0; i < 12; i++) sd.push_tri(mtl, v[f[i][0]], v[f[i][1]], v[f[i][2]]);
}

float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

}  // namespace

// addCornellBox, rayTracing.cpp:453-547
extern "C" int rt2_sd_add_cornell_box(rt2_scene_data* sd, float lightSize, float pad, int32_t lightMtl,
                                      int32_t lightEnabled) {
    return guard([&]() -> int {
        if (!sd) throw std::runtime_error("null scene data");
        Padded p = padded_box(*sd, pad);
        V3 c[8];
        box_corners(p, c);
        V3 boxSize = V3(p.maxX, p.maxY, p.maxZ) - V3(p.minX, p.minY, p.minZ);
        float centerX = (p.maxX + p.minX) / 2.0f;
        float centerZ = (p.maxZ + p.minZ) / 2.0f;
        float lMinX = centerX - lightSize * boxSize.x / 2.0f;
        float lMaxX = centerX + lightSize * boxSize.x / 2.0f;
        float lMinZ = centerZ - lightSize * boxSize.z / 2.0f;
        float lMaxZ = centerZ + lightSize * boxSize.z / 2.0f;
        float lY = p.maxY - 1e-3f;
        V3 l[4] = {V3(lMinX, lY, lMaxZ), V3(lMaxX, lY, lMaxZ), V3(lMinX, lY, lMinZ), V3(lMaxX, lY, lMinZ)};
        static const int walls[12][3] = {{0, 3, 1}, {0, 2, 3}, {0, 5, 4}, {0, 1, 5}, {0, 6, 2}, {0, 4, 6},
                                         {7, 1, 3}, {7, 5, 1}, {7, 2, 6}, {7, 3, 2}, {7, 4, 5}, {7, 6, 4}};
        static const int lights[4][3] = {{0, 3, 1}, {0, 2, 3}, {0, 1, 3}, {0, 3, 2}};
        for (int i = 0; i < 12; i++) sd->push_tri(0, c[walls[i][0]], c[walls[i][1]], c[walls[i][2]]);
        if (lightEnabled)
            for (int i = 0; i < 4; i++) sd->push_tri(lightMtl, l[lights[i][0]], l[lights[i][1]], l[lights[i][2]]);
        return 0;
    });
}

// addMirrorCornellBox, rayTracing.cpp:569-664
extern "C" int rt2_sd_add_mirror_cornell_box(rt2_scene_data* sd, float lightSize, float pad, int32_t lightMtl,
                                             int32_t mirrorMtl) {
    return guard([&]() -> int {
        if (!sd) throw std::runtime_error("null scene data");
        Padded p = padded_box(*sd, pad);
        V3 c[8];
        box_corners(p, c);
        float cx = (p.maxX + p.minX) / 2.0f;
        float cz = (p.maxZ + p.minZ) / 2.0f;
        float hs = lightSize * p.sceneSize.y / 2.0f;
        float off = 1e-3f;
        V3 l[4] = {V3(cx - hs, p.maxY - off, cz + hs), V3(cx + hs, p.maxY - off, cz + hs),
                   V3(cx - hs, p.maxY - off, cz - hs), V3(cx + hs, p.maxY - off, cz - hs)};
        static const int li[2][3] = {{0, 1, 2}, {1, 3, 2}};
        for (int i = 0; i < 12; i++) sd->push_tri(mirrorMtl, c[kWalls[i][0]], c[kWalls[i][1]], c[kWalls[i][2]]);
        for (int i = 0; i < 2; i++) sd->push_tri(lightMtl, l[li[i][0]], l[li[i][1]], l[li[i][2]]);
        return 0;
    });
}

// addSideLitCornellBox, rayTracing.cpp:690-847
extern "C" int rt2_sd_add_side_lit_cornell_box(rt2_scene_data* sd, float lightSize, float pad, int32_t lightMtl,
                                               int32_t wallMtl, int32_t rotate_) {
    return guard([&]() -> int {
        if (!sd) throw std::runtime_error("null scene data");
        Padded p = padded_box(*sd, pad);
        V3 c[8];
        box_corners(p, c);
        float cy = (p.maxY + p.minY) / 2.0f;
        float hs = lightSize * p.sceneSize.y / 2.0f;
        float off = 1e-3f;
        V3 a[4], b[4];
        static const int ia[2][3] = {{0, 2, 1}, {1, 2, 3}};
        static const int ib[2][3] = {{0, 1, 2}, {1, 3, 2}};
        if (!rotate_) {
            float cz = (p.maxZ + p.minZ) / 2.0f;
            a[0] = V3(p.minX + off, cy - hs, cz + hs);
            a[1] = V3(p.minX + off, cy + hs, cz + hs);
            a[2] = V3(p.minX + off, cy - hs, cz - hs);
            a[3] = V3(p.minX + off, cy + hs, cz - hs);
            b[0] = V3(p.maxX - off, cy - hs, cz + hs);
            b[1] = V3(p.maxX - off, cy + hs, cz + hs);
            b[2] = V3(p.maxX - off, cy - hs, cz - hs);
            b[3] = V3(p.maxX - off, cy + hs, cz - hs);
        } else {
            float cx = (p.maxX + p.minX) / 2.0f;
            a[0] = V3(cx - hs, cy - hs, p.maxZ - off);
            a[1] = V3(cx + hs, cy - hs, p.maxZ - off);
            a[2] = V3(cx - hs, cy + hs, p.maxZ - off);
            a[3] = V3(cx + hs, cy + hs, p.maxZ - off);
            b[0] = V3(cx - hs, cy - hs, p.minZ + off);
            b[1] = V3(cx + hs, cy - hs, p.minZ + off);
            b[2] = V3(cx - hs, cy + hs, p.minZ + off);
            b[3] = V3(cx + hs, cy + hs, p.minZ + off);
        }
        for (int i = 0; i < 12; i++) sd->push_tri(wallMtl, c[kWalls[i][0]], c[kWalls[i][1]], c[kWalls[i][2]]);
        for (int i = 0; i < 2; i++) sd->push_tri(lightMtl, a[ia[i][0]], a[ia[i][1]], a[ia[i][2]]);
        for (int i = 0; i < 2; i++) sd->push_tri(lightMtl, b[ib[i][0]], b[ib[i][1]], b[ib[i][2]]);
        return 0;
    });
}

// addSkyLightPlane, rayTracing.cpp:388-432 (the two triangles are appended twice)
extern "C" int rt2_sd_add_sky_light_plane(rt2_scene_data* sd, int32_t lightMtl) {
    return guard([&]() -> int {
        if (!sd) throw std::runtime_error("null scene data");
        Box b = sd->bounds();
        V3 s = b.size();
        float planeY = b.max.y + s.y * 0.3f;
        V3 k[4] = {V3(b.min.x, planeY, b.max.z), V3(b.max.x, planeY, b.max.z), V3(b.min.x, planeY, b.min.z),
                   V3(b.max.x, planeY, b.min.z)};
        static const int ki[2][3] = {{0, 3, 1}, {0, 2, 3}};
        for (int rep = 0; rep < 2; rep++)
            for (int i = 0; i < 2; i++) sd->push_tri(lightMtl, k[ki[i][0]], k[ki[i][1]], k[ki[i][2]]);
        return 0;
    });
}

// addCube, rayTracing.cpp:867-923
extern "C" int rt2_sd_add_cube(rt2_scene_data* sd, const float center[3], const float size[3],
                               const float rotation[3], int32_t mtl) {
    return guard([&]() -> int {
        if (!sd || !center || !size || !rotation) throw std::runtime_error("null argument");
        add_cube(*sd, V3(center[0], center[1], center[2]), V3(size[0], size[1], size[2]),
                 V3(rotation[0], rotation[1], rotation[2]), mtl);
        return 0;
    });
}

// createClassicCornellBox, rayTracing.cpp:949-1041
extern "C" int rt2_sd_create_classic_cornell_box(rt2_scene_data* sd, float roomSize, int32_t red, int32_t green,
                                                 int32_t white, int32_t light) {
    return guard([&]() -> int {
        if (!sd) throw std::runtime_error("null scene data");
        float half = roomSize * 0.5f;
        V3 c[8] = {V3(-half, -half, +half), V3(+half, -half, +half), V3(-half, +half, +half), V3(+half, +half, +half),
                   V3(-half, -half, -half), V3(+half, -half, -half), V3(-half, +half, -half), V3(+half, +half, -half)};
        struct W {
            int i[3];
            int m;
        };
        const W walls[12] = {{{0, 3, 1}, white}, {{0, 2, 3}, white}, {{4, 7, 6}, white}, {{4, 5, 7}, white},
                             {{0, 5, 4}, white}, {{0, 1, 5}, white}, {{2, 6, 7}, white}, {{2, 7, 3}, white},
                             {{0, 4, 6}, red},   {{0, 6, 2}, red},   {{1, 3, 7}, green}, {{1, 7, 5}, green}};
        for (const W& w : walls) sd->push_tri(w.m, c[w.i[0]], c[w.i[1]], c[w.i[2]]);
        float lw = roomSize * (130.0f / 555.0f);
        float ld = roomSize * (105.0f / 555.0f);
        float ly = half - 0.001f;
        V3 l[4] = {V3(-lw * 0.5f, ly, +ld * 0.5f), V3(+lw * 0.5f, ly, +ld * 0.5f), V3(-lw * 0.5f, ly, -ld * 0.5f),
                   V3(+lw * 0.5f, ly, -ld * 0.5f)};
        static const int li[2][3] = {{0, 2, 1}, {1, 2, 3}};
        for (int i = 0; i < 2; i++) sd->push_tri(light, l[li[i][0]], l[li[i][1]], l[li[i][2]]);
        float boxScale = 165.0f / 555.0f;
        float boxSize = roomSize * boxScale;
        float shortX = half * 0.5f, shortZ = -half * 0.3f;
        add_cube(*sd, V3(shortX, -half + boxSize * 0.5f, shortZ), V3(boxSize, boxSize, boxSize),
                 V3(0.0f, radians(-18.0f), 0.0f), white);
        float tallX = -half * 0.3f, tallZ = -half * 0.6f;
        float tallH = roomSize * (330.0f / 555.0f);
        add_cube(*sd, V3(tallX, -half + tallH * 0.5f, tallZ), V3(boxSize, tallH, boxSize),
                 V3(0.0f, radians(16.5f), 0.0f), white);
        return 0;
    });
}

// createDiverseCornellBox, rayTracing.cpp:1071-1118
extern "C" int rt2_sd_create_diverse_cornell_box(rt2_scene_data* sd, float roomSize, int32_t red, int32_t green,
                                                 int32_t white, int32_t light, int32_t glass, int32_t mirror,
                                                 int32_t checker, int32_t metal) {
    int rc = rt2_sd_create_classic_cornell_box(sd, roomSize, red, green, white, light);
    if (rc) return rc;
    return guard([&]() -> int {
        float half = roomSize * 0.5f;
        struct C {
            V3 p, s, r;
            int m;
        };
        const C cubes[9] = {
            {V3(-half * 0.7f, -half + 0.1f, half * 0.6f), V3(0.15f, 0.15f, 0.15f), V3(0.0f, 0.785f, 0.0f), glass},
            {V3(half * 0.6f, -half + 0.05f, -half * 0.4f), V3(0.08f, 0.08f, 0.08f), V3(0.2f, 0.5f, 0.3f), mirror},
            {V3(0.0f, -half + 0.2f, -half * 0.7f), V3(0.25f, 0.4f, 0.25f), V3(0.0f, 0.0f, 0.1f), checker},
            {V3(half * 0.3f, -half + 0.3f, half * 0.2f), V3(0.1f, 0.6f, 0.1f), V3(0.1f, 1.2f, 0.0f), metal},
            {V3(-half * 0.2f, -half + 0.15f, -half * 0.2f), V3(0.2f, 0.1f, 0.3f), V3(0.5f, 0.0f, 0.2f), glass},
            {V3(half * 0.8f, -half + 0.03f, half * 0.8f), V3(0.05f, 0.05f, 0.05f), V3(0.0f, 0.0f, 0.0f), mirror},
            {V3(half * 0.75f, -half + 0.08f, half * 0.75f), V3(0.06f, 0.06f, 0.06f), V3(0.3f, 0.3f, 0.3f), mirror},
            {V3(-half * 0.5f, -half + 0.02f, -half * 0.6f), V3(0.3f, 0.04f, 0.3f), V3(0.0f, 0.7f, 0.0f), checker},
            {V3(half * 0.1f, -half + 0.25f, half * 0.5f), V3(0.18f, 0.18f, 0.18f), V3(0.6f, 0.4f, 0.8f), metal},
        };
        for (const C& c : cubes) add_cube(*sd, c.p, c.s, c.r, c.m);
        return 0;
    });
}

/* ---- BVH, BVH.h:79-221 ------------------------------------------------------ */
namespace {

float node_cost(V3 size, int count) {
    float halfArea = size.x * (size.y + size.z) + size.y * size.z;
    return halfArea * (float)count;
}

struct BvhBuilder {
    SceneData& sd;
    std::vector<rt2_node>& nodes;
    static constexpr int kMaxDepth = 32;  // BVH.h:9

    static rt2_node make_node(const Box& b, int tri, int count, int child) {
        rt2_node n{};
        n.bmin[0] = b.min.x;
        n.bmin[1] = b.min.y;
        n.bmin[2] = b.min.z;
        n.bmax[0] = b.max.x;
        n.bmax[1] = b.max.y;
        n.bmax[2] = b.max.z;
        n.triangleIndex = tri;
        n.triangleCount = count;
        n.childIndex = child;
        return n;
    }
    static Box box_of(const rt2_node& n) {
        Box b;
        b.min = V3(n.bmin[0], n.bmin[1], n.bmin[2]);
        b.max = V3(n.bmax[0], n.bmax[1], n.bmax[2]);
        return b;
    }

    // evaluateSplit, BVH.h:92-115
    float evaluate(const rt2_node& node, int axis, float pos) const {
        Box a, b;
        int na = 0, nb = 0;
        for (int i = node.triangleIndex; i < node.triangleIndex + node.triangleCount; i++) {
            const BvhTri& t = sd.btris[i];
            if (t.center[axis] < pos) {
                a.grow(t);
                na++;
            } else {
                b.grow(t);
                nb++;
            }
        }
        return node_cost(a.size(), na) + node_cost(b.size(), nb);
    }

    // chooseSplit, BVH.h:117-143
    void choose(const rt2_node& node, int& axisOut, float& posOut, float& costOut) const {
        const int tests = 10;
        costOut = 1e32f;
        posOut = 0.0f;
        axisOut = 0;
        for (int axis = 0; axis < 3; axis++) {
            float s = node.bmin[axis], e = node.bmax[axis];
            for (int i = 0; i < tests; i++) {
                float t = (float)(i + 1) / (float)(tests + 1);
                float pos = s + (e - s) * t;
                float c = evaluate(node, axis, pos);
                if (c < costOut) {
                    costOut = c;
                    posOut = pos;
                    axisOut = axis;
                }
            }
        }
    }

    // BVH::split, BVH.h:170-220
    void split(int root, int depth) {
        if (depth == kMaxDepth || nodes[root].triangleCount < 1) return;
        int axis;
        float pos, cost;
        choose(nodes[root], axis, pos, cost);
        if (cost >= node_cost(box_of(nodes[root]).size(), nodes[root].triangleCount)) return;
        Box ba, bb;
        int aIdx = nodes[root].triangleIndex, aCnt = 0;
        int bIdx = nodes[root].triangleIndex, bCnt = 0;
        const int begin = nodes[root].triangleIndex, end = begin + nodes[root].triangleCount;
        for (int i = begin; i < end; i++) {
            bool inA = sd.btris[i].center[axis] < pos;
            if (inA) {
                ba.grow(sd.btris[i]);
                aCnt++;
                int sw = aIdx + aCnt - 1;
                std::swap(sd.btris[i], sd.btris[sw]);
                std::swap(sd.tris[i], sd.tris[sw]);
                bIdx += 1;
            } else {
                bb.grow(sd.btris[i]);
                bCnt++;
            }
        }
        ba.expand();
        bb.expand();
        if (aCnt > 0 || bCnt > 0) {
            int childA = (int)nodes.size();
            nodes[root].childIndex = childA;
            nodes.push_back(make_node(ba, aIdx, aCnt, -1));
            nodes.push_back(make_node(bb, bIdx, bCnt, -1));
            split(childA, depth + 1);
            split(childA + 1, depth + 1);
        }
    }
};

}  // namespace

extern "C" int rt2_sd_build_bvh(rt2_scene_data* sd) {
    return guard([&]() -> int {
        if (!sd) throw std::runtime_error("null scene data");
        sd->nodes.clear();
        Box b = sd->bounds();
        b.expand();
        sd->nodes.push_back(BvhBuilder::make_node(b, 0, (int)sd->tris.size(), -1));
        BvhBuilder bld{*sd, sd->nodes};
        bld.split(0, 1);
        return 0;
    });
}
