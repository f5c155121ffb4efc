/*
 * rt2.h — C-ABI of the MI355X-native render path (drop-in for the reference's
 * GL compute dispatch of RayTracing/Assets/Shaders/compute.glsl).
 *
 * Every entry point below replaces one piece of the reference's GPU boundary
 * (SURVEY.md §8b).  POD layouts are byte-identical to the reference's host
 * structs so a caller can hand over the very vectors it used to pass to
 * glBufferData:
 *
 *   rt2_triangle  == RTXTriangle      RayTracing/Assets/headers/mesh.h:112-139   (80 B)
 *   rt2_material  == Material         RayTracing/Assets/headers/mesh.h:26-103    (96 B)
 *   rt2_node      == Node             RayTracing/Assets/headers/BVH.h:54-65      (48 B)
 *   rt2_uniforms  == GlobalUniforms   RayTracing/Assets/headers/camera.h:10-36   (192 B, std140)
 *
 * Status convention: 0 = ok, < 0 = error; rt2_last_error() returns a
 * thread-local message.  No C++ exception crosses this ABI.
 *
 * Two groups of functions:
 *   (1) device path  (rt2_scene_*, rt2_render*, rt2_resolve_*) — HIP on gfx950;
 *   (2) host surface (rt2_sd_*, rt2_camera_*, rt2_write_png) — the reference's
 *       OBJ/MTL loader, Cornell-box builders, BVH build, camera and PNG writer,
 *       restated in C++ behind the same ABI.
 */
#ifndef RT2_H
#define RT2_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT2_ABI_VERSION 4

/* Material types: mesh.h:16-22 == compute.glsl:7-13 */
enum {
    RT2_DIFFUSE = 0,
    RT2_SPECULAR = 1,
    RT2_LIGHT = 2,
    RT2_CHECKER = 3,
    RT2_GLASS = 4,
    RT2_TEXTURE = 5,
    RT2_GLASS_HIGHLIGHT = 6
};

typedef struct rt2_vec4 { float x, y, z, w; } rt2_vec4;
typedef struct rt2_vec2 { float x, y; } rt2_vec2;

/* RTXTriangle, mesh.h:112-139.  GLSL std430 `Triangle` (compute.glsl:46-56)
 * reads a/b/c at byte 0/16/32, the UVs at 48/56/64 and mtlIndex at 72. */
typedef struct rt2_triangle {
    rt2_vec4 a, b, c;
    rt2_vec2 aTex, bTex, cTex;
    int32_t materialIndex;
    float pad;
} rt2_triangle;

/* Material, mesh.h:26-103 == compute.glsl:17-37 */
typedef struct rt2_material {
    rt2_vec4 color;
    rt2_vec4 specularColor;
    rt2_vec4 emissionColor;
    int32_t textureIndex;
    float emissionStrength;
    float smoothness;
    float specularProbability;
    float checkerScale;
    float refractiveIndex;
    int32_t materialType;
    int32_t index;
    int32_t isEdgeHighlight;
    int32_t pad1, pad2, pad3;
} rt2_material;

/* Node + BoundingBox, BVH.h:11-65 == compute.glsl:58-73 */
typedef struct rt2_node {
    float bmin[3];
    float pad0;
    float bmax[3];
    float pad1;
    int32_t triangleIndex;
    int32_t triangleCount;
    int32_t childIndex;
    int32_t pad;
} rt2_node;

/* GlobalUniforms, camera.h:10-36 == compute.glsl:119-146 (std140) */
typedef struct rt2_uniforms {
    int32_t pad;
    int32_t numTextures;
    uint32_t width;
    uint32_t height;
    int32_t numSpheres;
    int32_t numTriangles;
    int32_t basicShading;
    int32_t basicShadingShadow;
    rt2_vec4 basicShadingLightPosition;
    int32_t environmentalLight;
    int32_t maxBounceCount;
    int32_t numRaysPerPixel;
    uint32_t frameIndex;
    rt2_vec4 cameraPos;
    rt2_vec4 viewportRight;
    rt2_vec4 viewportUp;
    rt2_vec4 viewportFront;
    rt2_vec4 pixelRight;
    rt2_vec4 pixelUp;
    rt2_vec4 defocusDiskRight;
    rt2_vec4 defocusDiskUp;
} rt2_uniforms;

/* Image-row shard: the rows y in [0, height) with
 *   (y / tile_rows) % nranks == rank
 * in increasing order form this rank's slab (SURVEY.md §8e, row-tile
 * interleave).  {1, 0, 1} is the whole image. */
typedef struct rt2_shard {
    int32_t tile_rows;
    int32_t rank;
    int32_t nranks;
} rt2_shard;

/* Work counters of the last render on a scene (SURVEY.md §8d units). */
typedef struct rt2_stats {
    uint64_t samples;   /* pixel-rays traced = pixels * R * F              */
    uint64_t segments;  /* closest-hit queries (bounces actually traced)     */
    uint64_t tests;     /* ray-triangle tests = segments * N (brute force);
                           leaf tests (BVH traversal)                        */
    uint64_t node_visits; /* BVH traversal: interior nodes popped (box pairs
                             tested); 0 for brute force                      */
} rt2_stats;

/* An 8-bit image as stb_image returns it: `channels` (1..4) interleaved
 * bytes per pixel, rows of width*channels bytes, row 0 first in memory. */
typedef struct rt2_image {
    int32_t width;
    int32_t height;
    int32_t channels;
    uint8_t* pixels;
} rt2_image;

const char* rt2_last_error(void);
int rt2_abi_version(void);

/* ------------------------------------------------------------------------
 * (1) Device path
 * ---------------------------------------------------------------------- */

typedef struct rt2_scene rt2_scene;

/* Replaces the three SSBO uploads (rayTracing.cpp:1323-1325, SSBO.cpp:3-10,
 * glBufferData GL_STATIC_DRAW: the arrays are copied, the caller keeps
 * ownership).  `nodes` may be NULL (brute-force traversal does not need it).
 * Materials with materialType TEXTURE sample the images given to
 * rt2_scene_set_textures (getTriangleTextureColor, compute.glsl:342-368);
 * until that call they read black, as compute.glsl:349-350 does for a
 * texture index outside numTextures. */
int rt2_scene_create(const rt2_triangle* tris, int32_t n_tris,
                     const rt2_material* mats, int32_t n_mats,
                     const rt2_node* nodes, int32_t n_nodes,
                     int32_t device, rt2_scene** out);
void rt2_scene_destroy(rt2_scene* scene);

/* Number of slab rows a shard owns for an image of `height` rows. */
int32_t rt2_shard_rows(int32_t height, rt2_shard shard);
/* Image row y of slab row `local_row` (inverse of the interleave). */
int32_t rt2_shard_row(int32_t local_row, rt2_shard shard);

/* Replaces `frame_count` consecutive glDispatchCompute calls of compute.glsl
 * (rayTracing.cpp:184-191, uniforms->frameIndex = frame_begin + i), restricted
 * to the shard's rows, with the per-frame rgba32f imageStore (compute.glsl:700)
 * folded into an accumulator instead of a texture:
 *
 *   d_accum[4*(slab_row*W + x) + c] += color_f[c]   for f = frame_begin ...
 *
 * in increasing frame order (so splitting the frames over several calls gives
 * bit-identical sums).  d_accum is DEVICE memory of rows*W*4 floats.
 * d_accum8 (nullable, device, rows*W*4 uint32) accumulates the per-frame GL
 * unorm8 quantisation of the same colours — the reference screenshot path
 * (rayTracing.cpp:217-238).  `stream` is a hipStream_t (NULL = default);
 * the call is asynchronous like glDispatchCompute.  uniforms->basicShading != 0
 * selects the one-ray preview (traceBasic, compute.glsl:565-645 and the
 * basicShading branch of main, :672-678): deterministic, no jitter, no
 * tonemap; numRaysPerPixel is then ignored. */
int rt2_render(rt2_scene* scene, const rt2_uniforms* uniforms,
               uint32_t frame_begin, uint32_t frame_count, rt2_shard shard,
               float* d_accum, uint32_t* d_accum8, void* stream);

/* Blocking convenience wrapper — the readback half of screenshot()
 * (glReadPixels, rayTracing.cpp:217): renders into device buffers the scene
 * keeps between calls (allocated on first use, freed by rt2_scene_destroy), on
 * a stream of its own, and copies the resolved mean image back to host memory;
 * it waits for that stream only.  out_rgba (nullable):
 * rows*W*4 floats, mean over the frames (alpha = 1), slab-row order, slab row
 * 0 = lowest image row (GL convention, row 0 = bottom).  out_rgb8 (nullable):
 * rows*W*3 bytes, the reference's 8-bit screenshot average
 * (rayTracing.cpp:248-250), NOT flipped. */
int rt2_render_host(rt2_scene* scene, const rt2_uniforms* uniforms,
                    uint32_t frame_begin, uint32_t frame_count, rt2_shard shard,
                    float* out_rgba, uint8_t* out_rgb8);

/* Device resolve: out[i] = accum[i] / frames (rgb), alpha = 1.  Async. */
int rt2_resolve_rgba32f(const float* d_accum, int64_t n_pixels, uint32_t frames,
                        float* d_out, void* stream);
/* Host resolve of the 8-bit reference path (rayTracing.cpp:248-250):
 * u8(min(255, float(sum)/frames)) per channel, rgba sums -> rgb bytes. */
int rt2_resolve_rgb8_reference(const uint32_t* accum8, int64_t n_pixels, uint32_t frames,
                               uint8_t* out_rgb);

/* ------------------------------------------------------------------------
 * (1b) Multi-GPU: row-tile shards + one RCCL gather
 *
 * The reference renders on one GPU and reads the framebuffer back with
 * glReadPixels inside screenshot() (rayTracing.cpp:124-283, :217).  With N
 * ranks (one process per GPU), rank r renders the rows of rt2_shard
 * {tile_rows, r, N} and ONE ncclGather (RCCL over xGMI) brings the resolved
 * slabs to the root, which un-interleaves them: bit-identical to one GPU.
 *
 * Failure contract (raytracing2-fork_amd/csrc/device/rt2_comm_protocol.h):
 * every rank issues the same collectives in the same order.  A rank-local
 * failure (arguments, a shard that does not match the communicator, device
 * memory, a failed render) is decided by an agreement step — a 2-int
 * ncclAllReduce(max) read back on the host — before any gather, so every
 * rank returns < 0 and no gather is issued.  A rank that cannot take part in
 * an agreement (its communicator was aborted, the agreement's own copy or
 * allreduce fails) aborts and returns; its peers wait for it at most
 * RT2_COMM_TIMEOUT_S seconds (default 600; every host wait on a collective is
 * a poll of the stream and ncclCommGetAsyncError with that deadline), then
 * abort their communicator and return < 0.  An aborted owned communicator is
 * unusable: destroy it.  A wrapped communicator is never aborted here (its
 * owner must abort it); the handle only refuses further use.
 * RT2_FAULT_AT=<site>[@rank] injects a failure (tests only; sites
 * gather.prepare, gather.issue, check, render, agree.copy).
 * ---------------------------------------------------------------------- */
#define RT2_COMM_ID_BYTES 128 /* sizeof(ncclUniqueId) */
typedef struct rt2_comm rt2_comm;

/* ncclGetUniqueId: called once (by the root); the bytes travel to the other
 * ranks by any channel (a file, a socket, an MPI broadcast). */
int rt2_comm_unique_id(uint8_t* id /* RT2_COMM_ID_BYTES */);
/* ncclCommInitRank on `device` (blocks until all nranks have joined). */
int rt2_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, rt2_comm** out);
/* Uses a caller-owned ncclComm_t (not destroyed by rt2_comm_destroy). */
int rt2_comm_wrap(void* nccl_comm, int32_t device, rt2_comm** out);
void rt2_comm_destroy(rt2_comm* comm);
int rt2_comm_size(rt2_comm* comm, int32_t* nranks, int32_t* rank);
/* ncclCommGetAsyncError: < 0 (with rt2_last_error) if a collective failed. */
int rt2_comm_check(rt2_comm* comm);

/* Gathers every rank's slab — rt2_shard_rows(height, shard) rows of `width`
 * 16-byte pixels (an rgba32f image or the uint32x4 8-bit sums), device memory —
 * to `root` with one ncclGather and un-interleaves it there into d_image
 * (height*width pixels, device; ignored on other ranks).  shard.rank/nranks
 * must be the communicator's.  The host first waits for the work already
 * queued on `stream` (this rank's render: no peer is involved, so no deadline
 * applies; bounded at 20 x RT2_COMM_TIMEOUT_S, and twice its duration is added
 * to the deadlines that follow), then the ranks agree that each of them can
 * take part (one agreement step on the communicator's own stream, which could
 * not start on a device still busy with the render); the gather and the
 * un-interleave are then asynchronous on `stream`.  A local failure (a root without d_image, a
 * shard that does not match, no device memory) makes every rank return < 0
 * with nothing issued.  Once the gather is queued, a peer that fails inside
 * it (ncclCommAbort does not release ranks already in the collective) leaves
 * `stream` waiting: wait for it with rt2_comm_wait, not an unbounded
 * hipStreamSynchronize. */
int rt2_gather_slabs(rt2_comm* comm, const void* d_slab, int32_t width, int32_t height, rt2_shard shard,
                     int32_t root, void* d_image, void* stream);
/* The host waits for `stream` (e.g. rt2_gather_slabs' gather) under the
 * RT2_COMM_TIMEOUT_S deadline, polling ncclCommGetAsyncError: 0 when it has
 * drained; on a timeout, an RCCL error or a stream error the communicator is
 * aborted as above and < 0 returned (replaces the caller's
 * hipStreamSynchronize / cudaStreamSynchronize after the collective).  When
 * the last rt2_gather_slabs of this communicator was queued on `stream`, the
 * work queued before that gather (already waited for by rt2_gather_slabs) is
 * excluded from the deadline in the same way. */
int rt2_comm_wait(rt2_comm* comm, void* stream);
/* The root's un-interleave alone: d_gathered = [nranks][max_rows][width]
 * 16-byte pixels (rank-major slabs, padded to max_rows rows) -> d_image
 * [height][width] for the tile layout {tile_rows, -, nranks}.  Async. */
int rt2_unshard_slabs(const void* d_gathered, int32_t max_rows, int32_t width, int32_t height, rt2_shard layout,
                      void* d_image, void* stream);
/* rt2_render_host across ranks: every rank renders its shard, the resolved
 * slabs (and, if out_rgb8, the 8-bit sums) are gathered to `root`, which
 * receives the whole image in out_rgba (height*width*4 floats) / out_rgb8
 * (height*width*3 bytes, not flipped); other ranks' output pointers are
 * ignored.  Blocking; every rank must call it.  The 8-bit sums are accumulated
 * and gathered when ANY rank passes out_rgb8 (so ranks may pass different
 * pointers), and the ranks agree before the gather that every one of them
 * rendered (two agreement steps): a rank-local failure makes every rank
 * return < 0 ("a peer rank failed") instead of leaving peers blocked in the
 * gather.  The host waits for the gathers under the RT2_COMM_TIMEOUT_S
 * deadline before the root copies the image out. */
int rt2_render_host_gather(rt2_scene* scene, const rt2_uniforms* uniforms, uint32_t frame_begin,
                           uint32_t frame_count, rt2_shard shard, rt2_comm* comm, int32_t root,
                           float* out_rgba, uint8_t* out_rgb8);

/* Counters of the renders issued on this scene since the last reset
 * (synchronises the scene's device). */
int rt2_scene_stats(rt2_scene* scene, rt2_stats* out, int reset);

/* Kernel-variant control for experiments: 0 = auto.  Returns the variant the
 * next render will use for this scene. */
int rt2_scene_set_variant(rt2_scene* scene, int variant);

/* Closest-hit algorithm.  BRUTE (default): every triangle in array order, the
 * north-star kernel.  BVH: the reference's own traversal of the node array
 * (calculateRayCollisionBVH, compute.glsl:410-460; needs `nodes` at
 * rt2_scene_create) — identical to BRUTE except on exact distance ties, where
 * it resolves in the reference's visiting order. */
enum { RT2_TRAVERSAL_BRUTE = 0, RT2_TRAVERSAL_BVH = 1 };
int rt2_scene_set_traversal(rt2_scene* scene, int traversal);

/* Work-item shape for frame_count > 1 (default 1): the render hands out
 * (frame, pixel) items frame-major and adds the frames in order afterwards,
 * instead of one whole pixel (all frames) per item — a shorter tail at the end
 * of each launch.  Results are bit-identical either way; costs
 * frame_count * pixels * 16 B of device scratch per scene. */
int rt2_scene_set_frame_split(rt2_scene* scene, int enable);

/* Work-item order (default 0 = raster order): when enabled, each render
 * records a per-pixel cost map of the scene's slab (item time in shader
 * clocks) and the next render of the same slab hands out runs of 64
 * neighbouring pixels most-expensive-first (a GPU counting sort), so the last
 * items of a launch are cheap ones — the reference's progressive renders of
 * one view repeat the same per-pixel costs.  Measured: −7 % time on config E
 * (heavy-tailed mirror paths), neutral to −2 % elsewhere.  Results are
 * bit-identical in any order.  Renders of one scene are always ordered among
 * themselves (a render waits for the scene's previous one on any stream). */
int rt2_scene_set_cost_order(rt2_scene* scene, int enable);

/* Replaces binding the loader's textures to units 0..4 (rayTracing.cpp:
 * 1315-1320; Texture2D(path), textureClass.cpp:55-104): the images are copied
 * to HBM as RGBA8 with GL's unpack of GL_RED/GL_RG/GL_RGB/GL_RGBA bytes
 * (4-byte row alignment, GL_UNPACK_ALIGNMENT's default) and the 1-channel
 * swizzle (r, r, r, 1).  TEXTURE materials then sample texture
 * `textureIndex` with GL_LINEAR + GL_REPEAT (getTriangleTextureColor,
 * compute.glsl:342-368): black when textureIndex is outside [0,
 * uniforms->numTextures), magenta for an index >= 5 (the shader binds five
 * samplers), black for an index with no image here (an unbound unit).
 * n = 0 removes the textures. */
int rt2_scene_set_textures(rt2_scene* scene, const rt2_image* images, int32_t n);

/* ------------------------------------------------------------------------
 * (2) Host surface
 * ---------------------------------------------------------------------- */

/* Scene data under construction: the reference's rtxTriangles, bvhTriangles,
 * materials, texture list and BVH nodes (rayTracing.cpp:1256-1293). */
typedef struct rt2_scene_data rt2_scene_data;

rt2_scene_data* rt2_sd_create(void);
void rt2_sd_destroy(rt2_scene_data* sd);

/* getTrianglesData_ (mesh.h:279-613): first *.obj of the folder, every *.mtl
 * of the folder, every file of <folder>/textures decoded as a texture (in
 * directory order, flipped vertically on load, like Texture2D(path)).
 * Appends. */
int rt2_sd_load_obj_folder(rt2_scene_data* sd, const char* folder);
/* Decoded texture i of the scene data (pixels owned by sd) or < 0. */
int rt2_sd_texture(const rt2_scene_data* sd, int32_t i, rt2_image* out_view);

/* stbi_set_flip_vertically_on_load(flip); stbi_load(path, &w, &h, &n, 0)
 * (external/stb/stb_image.h v2.30 as Texture2D uses it), restated: PNG (all
 * depths/colour types, tRNS, interlace) and sequential-Huffman JPEG.  The
 * pixels are malloc'ed; release them with rt2_image_free. */
int rt2_image_load(const char* path, int32_t flip_vertically, rt2_image* out);
void rt2_image_free(rt2_image* image);
/* Appends one material; returns its index or < 0. */
int32_t rt2_sd_add_material(rt2_scene_data* sd, const rt2_material* m);
/* Appends one triangle (and its BVH triangle) as a builder would. */
int rt2_sd_add_triangle(rt2_scene_data* sd, const float a[3], const float b[3], const float c[3],
                        int32_t material_index);

/* Appends n complete triangle records (rtxTriangles.push_back). */
int rt2_sd_add_triangles(rt2_scene_data* sd, const rt2_triangle* tris, int32_t n);

/* Scene builders of rayTracing.cpp. */
int rt2_sd_add_cornell_box(rt2_scene_data* sd, float light_size, float pad, int32_t light_mtl,
                           int32_t light_enabled);                           /* :453-547 */
int rt2_sd_add_mirror_cornell_box(rt2_scene_data* sd, float light_size, float pad,
                                  int32_t light_mtl, int32_t mirror_mtl);    /* :569-664 */
int rt2_sd_add_side_lit_cornell_box(rt2_scene_data* sd, float light_size, float pad,
                                    int32_t light_mtl, int32_t wall_mtl, int32_t rotate); /* :690-847 */
int rt2_sd_add_sky_light_plane(rt2_scene_data* sd, int32_t light_mtl);       /* :388-432 */
int rt2_sd_add_cube(rt2_scene_data* sd, const float center[3], const float size[3],
                    const float rotation[3], int32_t mtl);                   /* :867-923 */
int rt2_sd_create_classic_cornell_box(rt2_scene_data* sd, float room, int32_t red, int32_t green,
                                      int32_t white, int32_t light);         /* :949-1041 */
int rt2_sd_create_diverse_cornell_box(rt2_scene_data* sd, float room, int32_t red, int32_t green,
                                      int32_t white, int32_t light, int32_t glass, int32_t mirror,
                                      int32_t checker, int32_t metal);       /* :1071-1118 */

/* BVH(bvhTriangles, rtxTriangles) (BVH.h:145-221): builds the node array and
 * reorders the triangles in place, exactly as the reference does. */
int rt2_sd_build_bvh(rt2_scene_data* sd);

int32_t rt2_sd_num_triangles(const rt2_scene_data* sd);
int32_t rt2_sd_num_materials(const rt2_scene_data* sd);
int32_t rt2_sd_num_nodes(const rt2_scene_data* sd);
int32_t rt2_sd_num_textures(const rt2_scene_data* sd);
const rt2_triangle* rt2_sd_triangles(const rt2_scene_data* sd);
const rt2_material* rt2_sd_materials(const rt2_scene_data* sd);
const rt2_node* rt2_sd_nodes(const rt2_scene_data* sd);
/* BVHTriangle min/max/center (mesh.h:141-154), 9 floats per triangle. */
int rt2_sd_bvh_triangles(const rt2_scene_data* sd, float* out9);
/* Texture file name i (directory order, mesh.h:305-318) or NULL. */
const char* rt2_sd_texture_name(const rt2_scene_data* sd, int32_t i);

/* Material helpers of mesh.h:47-102 (fields the reference leaves
 * uninitialised are zero here). */
void rt2_material_default(rt2_material* m);
void rt2_material_make_diffuse(rt2_material* m, float r, float g, float b);
void rt2_material_make_light(rt2_material* m, float r, float g, float b, float strength);
void rt2_material_make_specular(rt2_material* m, float r, float g, float b,
                                float sr, float sg, float sb, float smooth, float prob);
void rt2_material_make_checker(rt2_material* m, float scale);
void rt2_material_make_glass(rt2_material* m, float r, float g, float b, float ior);

/* Camera(...) + updateUniforms (camera.h:99-192): fills the eight camera
 * vec4s of `u` (other fields untouched). */
typedef struct rt2_camera {
    int32_t width, height;
    float position[3];
    float hfov, pitch, yaw;
    float focus_distance, defocus_angle, zoom;
} rt2_camera;
/* Reference defaults (rayTracing.cpp:82-89) for a width x height screen. */
void rt2_camera_default(rt2_camera* cam, int32_t width, int32_t height);
int rt2_camera_uniforms(const rt2_camera* cam, rt2_uniforms* u);
/* Offline-render uniforms (rayTracing.cpp:146-153 + :1386-1400). */
void rt2_uniforms_offline(rt2_uniforms* u, int32_t width, int32_t height, int32_t max_bounce,
                          int32_t rays_per_pixel, int32_t num_triangles, int32_t num_textures);

/* stbi_write_png surface (rayTracing.cpp:264): 8-bit, comps 1..4. */
int rt2_write_png(const char* path, int32_t w, int32_t h, int32_t comps, const uint8_t* data,
                  int32_t stride_bytes);

#ifdef __cplusplus
}
#endif

#endif /* RT2_H */
