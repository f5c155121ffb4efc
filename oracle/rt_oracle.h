/*
 * rt_oracle.h — TEST INFRASTRUCTURE ONLY (see rt_oracle.c).  CPU restatement of
 * RayTracing/Assets/Shaders/compute.glsl.  Struct layouts mirror the
 * reference's host structs directly (not the product header), so the oracle
 * stays independent of the code it checks.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

/* RTXTriangle, mesh.h:112-139 (80 B) */
typedef struct {
    float a[4], b[4], c[4];
    float aTex[2], bTex[2], cTex[2];
    int32_t materialIndex;
    float pad;
} oracle_triangle;

/* Material, mesh.h:26-103 (96 B) */
typedef struct {
    float color[4], specularColor[4], emissionColor[4];
    int32_t textureIndex;
    float emissionStrength, smoothness, specularProbability, checkerScale, refractiveIndex;
    int32_t materialType, index, isEdgeHighlight, pad1, pad2, pad3;
} oracle_material;

/* Node, BVH.h:54-65 (48 B) */
typedef struct {
    float bmin[3], pad0, bmax[3], pad1;
    int32_t triangleIndex, triangleCount, childIndex, pad;
} oracle_node;

/* GlobalUniforms, camera.h:10-36 (192 B) */
typedef struct {
    int32_t pad, numTextures;
    uint32_t width, height;
    int32_t numSpheres, numTriangles, basicShading, basicShadingShadow;
    float basicShadingLightPosition[4];
    int32_t environmentalLight, maxBounceCount, numRaysPerPixel;
    uint32_t frameIndex;
    float cameraPos[4], viewportRight[4], viewportUp[4], viewportFront[4];
    float pixelRight[4], pixelUp[4], defocusDiskRight[4], defocusDiskUp[4];
} oracle_uniforms;

#ifdef __cplusplus
extern "C" {
#endif

/* Renders frames [frame_begin, frame_begin+frame_count) of the listed image
 * rows (row 0 = bottom, as gl_GlobalInvocationID.y).  out_accum (nullable):
 * n_rows*W*4 floats, per-pixel SUM over frames in frame order (alpha = frame
 * count).  out_acc8 (nullable): n_rows*W*4 uint32 sums of the per-frame GL
 * unorm8 quantisation.  mode 0 = brute force, 1 = BVH (needs nodes). */
int oracle_render(const oracle_triangle* tris, int32_t n_tris, const oracle_material* mats, int32_t n_mats,
                  const oracle_node* nodes, int32_t n_nodes, const oracle_uniforms* u, uint32_t frame_begin,
                  uint32_t frame_count, const int32_t* rows, int32_t n_rows, int32_t mode, int32_t threads,
                  float* out_accum, uint32_t* out_acc8, uint64_t* out_segments, uint64_t* out_tests);

/* Same, over an arbitrary pixel list px = n_px (x, y) pairs; outputs are
 * n_px*4 in list order (bounded CPU samples of large configs). */
int oracle_render_pixels(const oracle_triangle* tris, int32_t n_tris, const oracle_material* mats, int32_t n_mats,
                         const oracle_node* nodes, int32_t n_nodes, const oracle_uniforms* u, uint32_t frame_begin,
                         uint32_t frame_count, const int32_t* px, int64_t n_px, int32_t mode, int32_t threads,
                         float* out_accum, uint32_t* out_acc8, uint64_t* out_segments, uint64_t* out_tests);

/* Textures for TEXTURE materials (global to the library): n stb-layout
 * images, whn = (width, height, channels) triples.  n = 0 clears. */
int oracle_set_textures(const int32_t* whn, const uint8_t* const* pixels, int32_t n);

uint32_t oracle_pcg_next(uint32_t* state, float* out);
int oracle_ray_triangle(const float o[3], const float d[3], const oracle_triangle* t, float* dst);
void oracle_sky(const float d[3], float out[3]);
float oracle_tonemap_srgb(float x);
float oracle_pinned(int which, float x);

#ifdef __cplusplus
}
#endif

#endif
