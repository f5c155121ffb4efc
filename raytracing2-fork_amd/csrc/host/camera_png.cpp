// Camera -> GlobalUniforms (RayTracing/Assets/headers/camera.h:99-192), the
// offline-render uniform settings (RayTracing/src/rayTracing.cpp:146-153,
// :1386-1400) and the PNG writer surface (stbi_write_png, rayTracing.cpp:264).
#include <zlib.h>

#include <cstdio>
#include <cstring>

#include "host_internal.h"

using namespace rt2h;

namespace {
// math_util.h:8 — `const float PI = atan(1.0) * 4.0f;` (double, then float)
const float kPI = (float)(std::atan(1.0) * 4.0f);
}  // namespace

// rayTracing.cpp:82-89 camera globals
extern "C" void rt2_camera_default(rt2_camera* cam, int32_t width, int32_t height) {
    cam->width = width;
    cam->height = height;
    cam->position[0] = 0.0f;
    cam->position[1] = 5.0f;
    cam->position[2] = 10.0f;
    cam->hfov = kPI / 6;
    cam->pitch = 0.0f;
    cam->yaw = kPI / 2.0f;
    cam->focus_distance = 20.0f;
    cam->defocus_angle = 0.0f;
    cam->zoom = 1.0f;
}

// Camera(...) -> updateBasisVectors (:150-160) -> updateViewportVectors(0)
// (:163-180) -> updateUniforms (:182-192).  camera.h calls the unqualified
// cos/sin/exp of <math.h> on float arguments, i.e. the double versions; the
// results are rounded to float on assignment.  glm::tan is tanf.
extern "C" int rt2_camera_uniforms(const rt2_camera* cam, rt2_uniforms* u) {
    if (!cam || !u) {
        set_error("null argument");
        return -1;
    }
    const float scrWidth = (float)cam->width, scrHeight = (float)cam->height;
    const float aspect = (float)cam->width / (float)cam->height;
    const float zoomSensitivity = 0.1f;
    const V3 worldUp(0.0f, 1.0f, 0.0f);
    V3 front;
    front.x = (float)(::cos((double)cam->yaw) * ::cos((double)cam->pitch));
    front.y = (float)::sin((double)cam->pitch);
    front.z = (float)(::sin((double)cam->yaw) * ::cos((double)cam->pitch));
    front = gnormalize(front);
    V3 right = gnormalize(gcross(worldUp, front));
    V3 up = gnormalize(gcross(front, right));

    float h = std::tan(cam->hfov / 2);
    float viewportWidth = (float)((double)(2 * h) / ::exp((double)(cam->zoom * zoomSensitivity)));
    float viewportHeight = viewportWidth / aspect;
    V3 viewportRight = right * viewportWidth * cam->focus_distance;
    V3 viewportUp = up * viewportHeight * cam->focus_distance;
    V3 viewportFront = -front * cam->focus_distance;
    V3 pixelRight = viewportRight / scrWidth;
    V3 pixelUp = viewportUp / scrHeight;
    float defocusRadius = cam->focus_distance * std::tan(cam->defocus_angle / 2.0f);
    V3 defocusDiskRight = right * defocusRadius;
    V3 defocusDiskUp = up * defocusRadius;

    u->cameraPos = vec4(V3(cam->position[0], cam->position[1], cam->position[2]));
    u->viewportRight = vec4(viewportRight);
    u->viewportUp = vec4(viewportUp);
    u->viewportFront = vec4(viewportFront);
    u->pixelRight = vec4(pixelRight);
    u->pixelUp = vec4(pixelUp);
    u->defocusDiskRight = vec4(defocusDiskRight);
    u->defocusDiskUp = vec4(defocusDiskUp);
    return 0;
}

extern "C" void rt2_uniforms_offline(rt2_uniforms* u, int32_t width, int32_t height, int32_t maxBounce,
                                     int32_t raysPerPixel, int32_t numTriangles, int32_t numTextures) {
    std::memset(u, 0, sizeof(*u));
    u->numTextures = numTextures;
    u->width = (uint32_t)width;
    u->height = (uint32_t)height;
    u->numSpheres = 0;
    u->numTriangles = numTriangles;
    u->basicShading = 0;        // SCREENSHOT_BASIC_SHADING
    u->basicShadingShadow = 0;  // BASIC_SHADING_SHADOW
    u->basicShadingLightPosition = rt2_vec4{10.0f, 100.0f, 1.0f, 0.0f};
    u->environmentalLight = 1;  // SCREENSHOT_ENVIRONMENTAL_LIGHT
    u->maxBounceCount = maxBounce;
    u->numRaysPerPixel = raysPerPixel;
    u->frameIndex = 0;
    rt2_camera cam;
    rt2_camera_default(&cam, width, height);
    rt2_camera_uniforms(&cam, u);
}

/* ---- PNG -------------------------------------------------------------------- */
namespace {
void put_be32(std::vector<unsigned char>& v, uint32_t x) {
    v.push_back((unsigned char)(x >> 24));
    v.push_back((unsigned char)(x >> 16));
    v.push_back((unsigned char)(x >> 8));
    v.push_back((unsigned char)x);
}
void put_chunk(FILE* f, const char* type, const std::vector<unsigned char>& data) {
    std::vector<unsigned char> buf;
    put_be32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    uint32_t crc = (uint32_t)crc32(0L, buf.data() + 4, (uInt)(buf.size() - 4));
    put_be32(buf, crc);
    std::fwrite(buf.data(), 1, buf.size(), f);
}
}  // namespace

extern "C" int rt2_write_png(const char* path, int32_t w, int32_t h, int32_t comps, const uint8_t* data,
                             int32_t stride) {
    return guard([&]() -> int {
        if (!path || !data || w <= 0 || h <= 0 || comps < 1 || comps > 4)
            throw std::runtime_error("rt2_write_png: bad argument");
        if (stride <= 0) stride = w * comps;
        std::vector<unsigned char> raw;
        raw.reserve((size_t)h * ((size_t)w * comps + 1));
        for (int y = 0; y < h; y++) {
            raw.push_back(0);  // filter type None
            const uint8_t* row = data + (size_t)y * stride;
            raw.insert(raw.end(), row, row + (size_t)w * comps);
        }
        uLongf zlen = compressBound((uLong)raw.size());
        std::vector<unsigned char> z(zlen);
        if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK)
            throw std::runtime_error("zlib compress failed");
        z.resize(zlen);
        FILE* f = std::fopen(path, "wb");
        if (!f) throw std::runtime_error(std::string("cannot open ") + path);
        static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
        std::fwrite(sig, 1, 8, f);
        std::vector<unsigned char> ihdr;
        put_be32(ihdr, (uint32_t)w);
        put_be32(ihdr, (uint32_t)h);
        static const unsigned char ctype[5] = {0, 0, 4, 2, 6};
        ihdr.push_back(8);
        ihdr.push_back(ctype[comps]);
        ihdr.push_back(0);
        ihdr.push_back(0);
        ihdr.push_back(0);
        put_chunk(f, "IHDR", ihdr);
        put_chunk(f, "IDAT", z);
        put_chunk(f, "IEND", {});
        bool ok = std::fclose(f) == 0;
        if (!ok) throw std::runtime_error("write failed");
        return 0;
    });
}
