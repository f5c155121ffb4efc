// MI355X (gfx950) render path: the per-pixel Monte-Carlo loop of
// RayTracing/Assets/Shaders/compute.glsl:472-701 as persistent HIP kernels,
// plus the device half of the C-ABI (include/rt2.h).
//
// Unit of work ("item") = one pixel-frame of the shard: its numRaysPerPixel
// rays run in order on one lane, like one compute.glsl invocation (the rays of
// a pixel-frame share one sequential RNG stream, compute.glsl:668/683).
//
// Execution model:
//   - one lane = one item at a time; every loop iteration each lane traces ONE
//     segment (closest-hit query + scatter) of its current ray, and a lane
//     whose item ends is refilled from a global counter (one atomic per wave);
//   - closest hit: brute force over all triangles (rt2_sweep.h, rt2_brute.h)
//     or the reference BVH's traversal order (rt2_bvh.h); both bit-identical
//     to the CPU oracle under the numerics contract of rt2_math.h;
//   - traceBasic preview, frame accumulation, cost-ordered scheduling and the
//     8-bit resolve live in rt2_misc_kernels.h.
//
// The headers are parts of this one translation unit (anonymous namespace,
// included below in dependency order), split only for reading.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../../include/rt2.h"
#include "rt2_math.h"

using namespace rt2d;

#include "rt2_sweep.h"
#include "rt2_path.h"
#include "rt2_brute.h"
#include "rt2_mfma.h"
#include "rt2_k5_tiles.h"
#include "rt2_k5_resident.h"
#include "rt2_assist.h"
#include "rt2_bvh.h"
#include "rt2_misc_kernels.h"

/* =========================================================================
 * C-ABI, device half
 * ======================================================================= */
namespace rt2h {
void set_error(const std::string& msg);
}

#define HIPCHECK(expr)                                                                         \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            rt2h::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                \
            return -1;                                                                         \
        }                                                                                      \
    } while (0)

constexpr int kCounters = 32;  // [0] items, [1..7] stats + wave-end, [8..] kernel diagnostics
struct rt2_scene {
    int device = 0;
    int n_tris = 0, n_mats = 0, n_nodes = 0;
    rt2_triangle* d_raw = nullptr;
    float4* d_tri = nullptr;
    int* d_mtl = nullptr;
    rt2_material* d_mats = nullptr;
    rt2_node* d_nodes = nullptr;
    float4* d_recs = nullptr;                   // BVH v2 child-pair records
    float4* d_plk = nullptr;                    // sweep_plk filter records (4 float4 per triangle)
    int plk_ok = 0;                             // sweep_plk usable: <= 1/64 of the triangles outside its range
    int plk_outside = 0;                        // triangles with an always-pass record
    float plk_A = 0.0f;                         // max |a_i| over the triangles
    _Float16* d_mfma = nullptr;                 // render_mfma filter records (rt2_mfma.h)
    float* d_mfma_tau = nullptr;                // per-triangle record scale
    _Float16* d_mfma_k16 = nullptr;             // sweep_k16 records (32-triangle groups, 7 KiB each)
    float* d_mfma_k16_tau = nullptr;            // per-triangle record scale (same values as d_mfma_tau)
    float2* d_mfma_k16_bnd = nullptr;           // per-triangle m.z residual bounds of the 5-product form (k5)
    _Float16* d_mfma_kt = nullptr;              // kthr records (threshold in the K-slots: 4 KiB per 32 triangles)
    int mfma_ok = 0;                            // render_mfma usable (records built, scene in range)
    float mfma_A = 0.0f;                        // max |a_i| over the in-range triangles
    float4* d_fb = nullptr;                     // frame_split scratch (per-frame colours)
    uchar4* d_texels = nullptr;                 // textures, RGBA8
    int4* d_tex_desc = nullptr;
    int n_tex = 0;
    size_t fb_bytes = 0;
    int bvh_root = 0;                           // BVH v2 stack entry of node 0
    int recs_ok = 0;                            // BVH v3 fast-path precondition on the boxes
    int split_frames = 1;                       // frame-major (frame, pixel) items when F > 1
    unsigned long long frame_scratch_cap = 2ull << 30;  // bytes of per-frame planes per launch
    int cost_order = 0;                         // order items by the previous launch's per-pixel cost (opt-in)
    uint32_t* d_cost = nullptr;                 // per-pixel cost map of the last launch
    uint32_t* d_order = nullptr;                // pixel order for the next launch
    uint32_t* d_hist = nullptr;                 // 32 counters
    unsigned long long cost_npix = 0;           // pixels the cost map describes (0 = none)
    unsigned long long cost_cap = 0;
    int cost_key[4] = {0, 0, 0, 0};             // W, tile_rows, rank, nranks the map belongs to
    hipEvent_t last_launch = nullptr;           // renders of one scene are ordered (shared scratch)
    bool last_launch_valid = false;
    unsigned long long* d_counters = nullptr;  // [0] item counter, [1] segments
    unsigned long long samples = 0, tests_per_seg = 0;
    int variant = 0;
    int last_variant = -1;
    int traversal = RT2_TRAVERSAL_BRUTE;
    int bvh_depth = 0;              // longest root-to-leaf path (nodes)
    int last_kind = 0;              // kind of the last launch (stats: tests)
    unsigned long long diag[kCounters] = {};
    int num_cus = 256;
    size_t max_lds = 65536;
    // rt2_render_host: device buffers reused across calls (grown on demand,
    // freed with the scene) and the stream the blocking wrapper runs on
    hipStream_t host_stream = nullptr;
    float4* d_host_acc = nullptr;   // float accumulator
    float4* d_host_res = nullptr;   // resolved mean
    uint4* d_host_acc8 = nullptr;   // 8-bit path sums
    uint8_t* d_host_rgb8 = nullptr; // 8-bit path result (3 B per pixel)
    size_t host_cap = 0;            // pixels the four buffers hold
    unsigned long long* d_region_ctr = nullptr;  // 8 item-region counters, 128 B apart
    unsigned long long* wave_log = nullptr;  // diagnostic wave timeline (rt2_scene_set_wave_log)
    uint32_t wave_log_n = 0;
};

// Validates a reference node array (BVH.h layout) against the triangle count
// and returns its depth; < 0 on a malformed array (child out of range, cycle,
// leaf range outside the triangles).
static int bvh_depth_check(const rt2_node* nodes, int n_nodes, int n_tris, std::string& err) {
    if (n_nodes < 1) {
        err = "empty node array";
        return -1;
    }
    std::vector<int> depth(n_nodes, 0);
    std::vector<int> stack;
    stack.push_back(0);
    depth[0] = 1;
    int maxd = 1;
    long long visited = 0;
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        if (++visited > n_nodes) {
            err = "node graph is not a tree";
            return -1;
        }
        const rt2_node& n = nodes[i];
        if (n.childIndex == -1) {
            if (n.triangleCount > 0 && (n.triangleIndex < 0 || (long long)n.triangleIndex + n.triangleCount > n_tris)) {
                err = "leaf " + std::to_string(i) + " references triangles outside [0, " + std::to_string(n_tris) + ")";
                return -1;
            }
            continue;
        }
        if (n.childIndex <= 0 || n.childIndex + 1 >= n_nodes) {
            err = "node " + std::to_string(i) + " has child index " + std::to_string(n.childIndex) + " out of range";
            return -1;
        }
        for (int c = n.childIndex; c <= n.childIndex + 1; c++) {
            depth[c] = depth[i] + 1;
            maxd = std::max(maxd, depth[c]);
            stack.push_back(c);
        }
    }
    return maxd;
}

// Child-pair records for render_bvh2 (layout: see bvh_step).  Interior nodes
// are numbered in depth-first pre-order (parents before children, left
// subtree first) so records of a subtree are contiguous.
static int bvh_records(const rt2_node* nodes, int n_nodes, std::vector<float4>& rec, int& root, std::string& err) {
    if (n_nodes >= (1 << 26)) {
        err = "more than 2^26 nodes";
        return -1;
    }
    std::vector<int> rid(n_nodes, -1);
    int n_int = 0;
    std::vector<int> stack{0};
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        if (nodes[i].childIndex == -1) continue;
        rid[i] = n_int++;
        stack.push_back(nodes[i].childIndex + 1);
        stack.push_back(nodes[i].childIndex);
    }
    auto enc = [&](int i) -> int {
        const rt2_node& n = nodes[i];
        if (n.childIndex != -1) return rid[i];
        const int cnt = std::max(n.triangleCount, 0);
        const int start = cnt > 0 ? n.triangleIndex : 0;
        if (cnt <= 30 && start >= 0 && start < (1 << 26)) return ~((start << 5) | cnt);
        return ~((i << 5) | 31);
    };
    rec.assign((size_t)std::max(n_int, 1) * 4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (int i = 0; i < n_nodes; i++) {
        if (rid[i] < 0) continue;
        const rt2_node& A = nodes[nodes[i].childIndex];
        const rt2_node& B = nodes[nodes[i].childIndex + 1];
        float4* r = &rec[(size_t)rid[i] * 4];
        r[0] = make_float4(A.bmin[0], A.bmin[1], A.bmin[2], A.bmax[0]);
        r[1] = make_float4(A.bmax[1], A.bmax[2], B.bmin[0], B.bmin[1]);
        r[2] = make_float4(B.bmin[2], B.bmax[0], B.bmax[1], B.bmax[2]);
        int e[4] = {enc(nodes[i].childIndex), enc(nodes[i].childIndex + 1), 0, 0};
        std::memcpy(&r[3], e, sizeof(e));
    }
    root = enc(0);
    return n_int;
}

// GL's unpack of a tightly packed stb image (GL_UNPACK_ALIGNMENT 4: rows
// start every align4(w*n) bytes; bytes past the buffer read as 0 — the
// reference reads past its allocation there) into RGBA8, with the swizzles of
// Texture2D(path) (1 channel: r,r,r,1; GL_RG: r,g,0,1; GL_RGB: r,g,b,1).
static void gl_unpack_rgba8(const rt2_image& im, uchar4* out) {
    const size_t n = (size_t)im.channels, stride = ((size_t)im.width * n + 3) & ~(size_t)3;
    const size_t total = (size_t)im.width * im.height * n;
    auto at = [&](size_t i) -> uint8_t { return i < total ? im.pixels[i] : (uint8_t)0; };
    for (int j = 0; j < im.height; j++)
        for (int i = 0; i < im.width; i++) {
            const size_t b = (size_t)j * stride + (size_t)i * n;
            uchar4 t;
            if (n == 1) t = make_uchar4(at(b), at(b), at(b), 255);
            else if (n == 2) t = make_uchar4(at(b), at(b + 1), 0, 255);
            else if (n == 3) t = make_uchar4(at(b), at(b + 1), at(b + 2), 255);
            else t = make_uchar4(at(b), at(b + 1), at(b + 2), at(b + 3));
            out[(size_t)j * im.width + i] = t;
        }
}

extern "C" int rt2_scene_set_textures(rt2_scene* s, const rt2_image* images, int32_t n) {
    if (!s || n < 0 || (n > 0 && !images)) {
        rt2h::set_error("rt2_scene_set_textures: bad argument");
        return -1;
    }
    size_t total = 0;
    for (int i = 0; i < n; i++) {
        const rt2_image& im = images[i];
        if (im.width < 1 || im.height < 1 || im.channels < 1 || im.channels > 4 || !im.pixels) {
            rt2h::set_error("rt2_scene_set_textures: image " + std::to_string(i) + " is empty or has " +
                            std::to_string(im.channels) + " channels");
            return -1;
        }
        total += (size_t)im.width * im.height;
    }
    HIPCHECK(hipSetDevice(s->device));
    HIPCHECK(hipDeviceSynchronize());
    (void)hipFree(s->d_texels);
    (void)hipFree(s->d_tex_desc);
    s->d_texels = nullptr;
    s->d_tex_desc = nullptr;
    s->n_tex = 0;
    if (n == 0) return 0;
    std::vector<uchar4> host(total);
    std::vector<int4> desc(n);
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        gl_unpack_rgba8(images[i], host.data() + off);
        desc[i] = make_int4(images[i].width, images[i].height, (int)(uint32_t)(off & 0xffffffffu), (int)(off >> 32));
        off += (size_t)images[i].width * images[i].height;
    }
    HIPCHECK(hipMalloc(&s->d_texels, total * sizeof(uchar4)));
    HIPCHECK(hipMalloc(&s->d_tex_desc, n * sizeof(int4)));
    HIPCHECK(hipMemcpy(s->d_texels, host.data(), total * sizeof(uchar4), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(s->d_tex_desc, desc.data(), n * sizeof(int4), hipMemcpyHostToDevice));
    s->n_tex = n;
    return 0;
}

// Not in rt2.h (test hook): bytes of per-frame colour planes one launch may use.
extern "C" int rt2_scene_set_frame_scratch_cap(rt2_scene* s, unsigned long long bytes) {
    if (!s || bytes == 0) return -1;
    s->frame_scratch_cap = bytes;
    return 0;
}

extern "C" int rt2_scene_set_cost_order(rt2_scene* s, int enable) {
    if (!s) {
        rt2h::set_error("rt2_scene_set_cost_order: null scene");
        return -1;
    }
    s->cost_order = enable ? 1 : 0;
    s->cost_npix = 0;  // forget the map
    return 0;
}

// Not in rt2.h (diagnostics): the assist kernel writes a per-wave timeline
// {start, first item-less lane, end, segments} in 10-ns ticks to d_log
// (4 x u64 per wave, n waves; null turns it off).
extern "C" int rt2_scene_set_wave_log(rt2_scene* s, unsigned long long* d_log, uint32_t n) {
    if (!s) return -1;
    s->wave_log = d_log;
    s->wave_log_n = d_log ? n : 0;
    return 0;
}

extern "C" int rt2_scene_set_frame_split(rt2_scene* s, int enable) {
    if (!s) {
        rt2h::set_error("rt2_scene_set_frame_split: null scene");
        return -1;
    }
    s->split_frames = enable ? 1 : 0;
    return 0;
}

extern "C" int rt2_scene_set_traversal(rt2_scene* s, int traversal) {
    if (!s || (traversal != RT2_TRAVERSAL_BRUTE && traversal != RT2_TRAVERSAL_BVH)) {
        rt2h::set_error("rt2_scene_set_traversal: bad argument");
        return -1;
    }
    if (traversal == RT2_TRAVERSAL_BVH && s->n_nodes == 0) {
        rt2h::set_error("rt2_scene_set_traversal: BVH traversal needs the node array (rt2_scene_create nodes)");
        return -1;
    }
    s->traversal = traversal;
    return 0;
}

static int scene_init(rt2_scene* s, const rt2_triangle* tris, int32_t n_tris, const rt2_material* mats,
                      int32_t n_mats, const rt2_node* nodes, int32_t n_nodes, int32_t device);

extern "C" int rt2_scene_create(const rt2_triangle* tris, int32_t n_tris, const rt2_material* mats, int32_t n_mats,
                                const rt2_node* nodes, int32_t n_nodes, int32_t device, rt2_scene** out) {
    if (!out || n_tris < 0 || n_mats < 1 || !mats || (n_tris > 0 && !tris)) {
        rt2h::set_error("rt2_scene_create: bad argument");
        return -1;
    }
    for (int i = 0; i < n_tris; i++) {
        if (tris[i].materialIndex < 0 || tris[i].materialIndex >= n_mats) {
            rt2h::set_error("rt2_scene_create: triangle " + std::to_string(i) + " has material index " +
                            std::to_string(tris[i].materialIndex) + " outside [0, " + std::to_string(n_mats) + ")");
            return -1;
        }
    }
    int ndev = 0;
    HIPCHECK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) {
        rt2h::set_error("rt2_scene_create: no HIP device " + std::to_string(device));
        return -1;
    }
    HIPCHECK(hipSetDevice(device));
    rt2_scene* s = new rt2_scene();
    if (scene_init(s, tris, n_tris, mats, n_mats, nodes, n_nodes, device) != 0) {
        rt2_scene_destroy(s);  // frees whatever was allocated before the failure
        return -1;
    }
    *out = s;
    return 0;
}

// Uploads and derived device arrays of rt2_scene_create; on failure returns
// -1 with the error set and leaves the partial scene to the caller to destroy.
static int scene_init(rt2_scene* s, const rt2_triangle* tris, int32_t n_tris, const rt2_material* mats,
                      int32_t n_mats, const rt2_node* nodes, int32_t n_nodes, int32_t device) {
    s->device = device;
    s->n_tris = n_tris;
    s->n_mats = n_mats;
    s->n_nodes = nodes ? n_nodes : 0;
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, device));
    s->num_cus = prop.multiProcessorCount;
    s->max_lds = prop.maxSharedMemoryPerMultiProcessor ? prop.maxSharedMemoryPerMultiProcessor : 65536;
    const size_t nt = (size_t)std::max(n_tris, 1);
    HIPCHECK(hipMalloc(&s->d_raw, nt * sizeof(rt2_triangle)));
    HIPCHECK(hipMalloc(&s->d_tri, nt * 3 * sizeof(float4)));
    HIPCHECK(hipMalloc(&s->d_mtl, nt * sizeof(int)));
    HIPCHECK(hipMalloc(&s->d_mats, (size_t)n_mats * sizeof(rt2_material)));
    HIPCHECK(hipMalloc(&s->d_counters, kCounters * sizeof(unsigned long long)));
    HIPCHECK(hipMemset(s->d_counters, 0, kCounters * sizeof(unsigned long long)));
    if (n_tris > 0) HIPCHECK(hipMemcpy(s->d_raw, tris, (size_t)n_tris * sizeof(rt2_triangle), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(s->d_mats, mats, (size_t)n_mats * sizeof(rt2_material), hipMemcpyHostToDevice));
    if (s->n_nodes > 0) {
        std::string err;
        s->bvh_depth = bvh_depth_check(nodes, n_nodes, n_tris, err);
        if (s->bvh_depth < 0 || s->bvh_depth > 62) {
            if (s->bvh_depth > 62) err = "BVH deeper than compute.glsl's 64-entry stack";
            rt2h::set_error("rt2_scene_create: bad node array: " + err);
            return -1;
        }
        HIPCHECK(hipMalloc(&s->d_nodes, (size_t)n_nodes * sizeof(rt2_node)));
        HIPCHECK(hipMemcpy(s->d_nodes, nodes, (size_t)n_nodes * sizeof(rt2_node), hipMemcpyHostToDevice));
        std::vector<float4> rec;
        if (bvh_records(nodes, n_nodes, rec, s->bvh_root, err) < 0) {
            rt2h::set_error("rt2_scene_create: bad node array: " + err);
            return -1;
        }
        // the first three float4 of a record are box coordinates (the 4th: stack entries)
        s->recs_ok = 1;
        for (size_t i = 0; i < rec.size(); i++) {
            if (i % 4 == 3) continue;
            for (float c : {rec[i].x, rec[i].y, rec[i].z, rec[i].w})
                if (!(c == 0.0f || (std::fabs(c) >= 0x1p-37f && std::fabs(c) <= 0x1p59f))) s->recs_ok = 0;
        }
        HIPCHECK(hipMalloc(&s->d_recs, rec.size() * sizeof(float4)));
        HIPCHECK(hipMemcpy(s->d_recs, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice));
    }
    if (n_tris > 0) {
        hipLaunchKernelGGL(prep_triangles, dim3((n_tris + 255) / 256), dim3(256), 0, 0, s->d_raw, n_tris, s->d_tri,
                           s->d_mtl);
        HIPCHECK(hipGetLastError());
#ifdef RT2_EXPERIMENTS
        HIPCHECK(hipMalloc(&s->d_plk, nt * 4 * sizeof(float4)));
        // two scratch words in an unused counter slot (zeroed again below)
        uint32_t* d_flags = reinterpret_cast<uint32_t*>(s->d_counters + kCounters - 2);
        HIPCHECK(hipMemset(d_flags, 0, 2 * sizeof(uint32_t)));
        hipLaunchKernelGGL(prep_plk, dim3((n_tris + 255) / 256), dim3(256), 0, 0, s->d_tri, n_tris, s->d_plk, d_flags);
        HIPCHECK(hipGetLastError());
        uint32_t flags[2];
        HIPCHECK(hipMemcpy(flags, d_flags, sizeof(flags), hipMemcpyDeviceToHost));
        HIPCHECK(hipMemset(d_flags, 0, 2 * sizeof(uint32_t)));
        s->plk_outside = (int)flags[0];
        s->plk_ok = (unsigned long long)flags[0] * 64 <= (unsigned long long)n_tris;  // <= 1/64 always-pass records
        std::memcpy(&s->plk_A, &flags[1], sizeof(float));
#endif
        // matrix-core filter records in the k16 layout (sweep_k16 and its
        // 5-product form): 7 KiB per 32 triangles; the prep's flags give the
        // scene's largest |a_i|, the filter's range check.  (The 16x16x32
        // layout of the experiment variants and the probe's layout 0 is built
        // on first use: ensure_mfma16.)
        const int n_pad32 = (n_tris + 31) / 32 * 32;
        HIPCHECK(hipMalloc(&s->d_mfma_k16, (size_t)n_pad32 * kK16Ops * 16 * sizeof(_Float16)));
        HIPCHECK(hipMalloc(&s->d_mfma_k16_tau, (size_t)n_pad32 * sizeof(float)));
        HIPCHECK(hipMalloc(&s->d_mfma_k16_bnd, (size_t)n_pad32 * sizeof(float2)));
        uint32_t* d_mflags = reinterpret_cast<uint32_t*>(s->d_counters + kCounters - 2);
        HIPCHECK(hipMemset(d_mflags, 0, 2 * sizeof(uint32_t)));
        hipLaunchKernelGGL(prep_mfma_k16, dim3((n_pad32 + 255) / 256), dim3(256), 0, 0, s->d_tri, n_tris, n_pad32,
                           s->d_mfma_k16, s->d_mfma_k16_tau, s->d_mfma_k16_bnd, d_mflags);
        HIPCHECK(hipGetLastError());
        uint32_t mflags[2];
        HIPCHECK(hipMemcpy(mflags, d_mflags, sizeof(mflags), hipMemcpyDeviceToHost));
        HIPCHECK(hipMemset(d_mflags, 0, 2 * sizeof(uint32_t)));
        std::memcpy(&s->mfma_A, &mflags[1], sizeof(float));
        s->mfma_ok = s->mfma_A <= 0x1p20f;
        // the kthr records (rt2_mfma.h prep_mfma_kt: the threshold in the
        // K-slots), 4 KiB per 32 triangles; its flags duplicate the above
        HIPCHECK(hipMalloc(&s->d_mfma_kt, (size_t)n_pad32 * kKtOps * 16 * sizeof(_Float16)));
        hipLaunchKernelGGL(prep_mfma_kt, dim3((n_pad32 + 255) / 256), dim3(256), 0, 0, s->d_tri, n_tris, n_pad32,
                           s->d_mfma_kt, d_mflags);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemset(d_mflags, 0, 2 * sizeof(uint32_t)));
    }
    HIPCHECK(hipDeviceSynchronize());
    return 0;
}

// The 16x16x32 record layout (5 KiB per 16 triangles: the experiment
// variants of that form and the filter probe's layout 0), built on first use
// so that a product scene does not keep 320 B per triangle it never reads.
static int ensure_mfma16(rt2_scene* s) {
    if (s->d_mfma || s->n_tris <= 0) return 0;
    HIPCHECK(hipSetDevice(s->device));
    const int n_pad = (s->n_tris + 15) / 16 * 16;
    HIPCHECK(hipMalloc(&s->d_mfma, (size_t)n_pad * kMfmaQ * 32 * sizeof(_Float16)));
    HIPCHECK(hipMalloc(&s->d_mfma_tau, (size_t)n_pad * sizeof(float)));
    HIPCHECK(hipDeviceSynchronize());  // the scratch flags below are the counters' last two words
    uint32_t* d_mflags = reinterpret_cast<uint32_t*>(s->d_counters + kCounters - 2);
    HIPCHECK(hipMemset(d_mflags, 0, 2 * sizeof(uint32_t)));
    hipLaunchKernelGGL(prep_mfma, dim3((n_pad + 255) / 256), dim3(256), 0, 0, s->d_tri, s->n_tris, n_pad, s->d_mfma,
                       s->d_mfma_tau, d_mflags);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemset(d_mflags, 0, 2 * sizeof(uint32_t)));
    HIPCHECK(hipDeviceSynchronize());
    return 0;
}

extern "C" void rt2_scene_destroy(rt2_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipFree(s->d_raw);
    (void)hipFree(s->d_tri);
    (void)hipFree(s->d_mtl);
    (void)hipFree(s->d_mats);
    (void)hipFree(s->d_nodes);
    (void)hipFree(s->d_recs);
    (void)hipFree(s->d_plk);
    (void)hipFree(s->d_mfma);
    (void)hipFree(s->d_mfma_tau);
    (void)hipFree(s->d_mfma_k16);
    (void)hipFree(s->d_mfma_k16_tau);
    (void)hipFree(s->d_mfma_k16_bnd);
    (void)hipFree(s->d_mfma_kt);
    (void)hipFree(s->d_fb);
    (void)hipFree(s->d_cost);
    (void)hipFree(s->d_order);
    (void)hipFree(s->d_hist);
    if (s->last_launch) (void)hipEventDestroy(s->last_launch);
    (void)hipFree(s->d_texels);
    (void)hipFree(s->d_tex_desc);
    (void)hipFree(s->d_counters);
    (void)hipFree(s->d_host_acc);
    (void)hipFree(s->d_host_res);
    (void)hipFree(s->d_host_acc8);
    (void)hipFree(s->d_host_rgb8);
    (void)hipFree(s->d_region_ctr);
    if (s->host_stream) (void)hipStreamDestroy(s->host_stream);
    delete s;
}

extern "C" int32_t rt2_shard_rows(int32_t height, rt2_shard sh) {
    if (sh.tile_rows < 1 || sh.nranks < 1 || sh.rank < 0 || sh.rank >= sh.nranks || height < 0) return -1;
    int32_t n = 0;
    for (int32_t t = sh.rank; (int64_t)t * sh.tile_rows < height; t += sh.nranks)
        n += std::min(sh.tile_rows, height - t * sh.tile_rows);
    return n;
}

extern "C" int32_t rt2_shard_row(int32_t local_row, rt2_shard sh) {
    int32_t t = local_row / sh.tile_rows;
    return (t * sh.nranks + sh.rank) * sh.tile_rows + local_row % sh.tile_rows;
}


namespace {
constexpr int kTileTris = 1024;  // 48 KiB of LDS per tile

// Kernel variants (rt2_scene_set_variant).  Ids are stable across builds: the
// product build carries the variants the launcher chooses automatically; the
// A/B experiments measured in DESIGN.md ("Tried and measured") are compiled
// only with -DRT2_EXPERIMENTS (make EXPERIMENTS=1).
enum Kind : int {
    K_RESIDENT = 0, K_TILED = 1, K_SMEM = 2, K_SPLIT = 3, K_ASSIST = 4, K_MFMA = 9, K_MASSIST = 10,  // brute force
    K_BVH = 5, K_BVH2 = 6, K_BVH3 = 7, K_BVH4 = 8                                     // BVH (kind >= K_BVH)
};
struct Variant {
    int id;
    int kind;
    int block;
    hipError_t (*launch)(const RenderParams&, int blocks, size_t lds, hipStream_t st);
    const void* kernel;
    const char* name;
};

template <auto K, int BLOCK>
hipError_t launch_k(const RenderParams& p, int blocks, size_t lds, hipStream_t st) {
    hipLaunchKernelGGL(K, dim3(blocks), dim3(BLOCK), lds, st, p);
    return hipGetLastError();
}
#define RT2_VARIANT(ID, KIND, KERNEL, BLOCK, NAME) \
    Variant { ID, KIND, BLOCK, launch_k<KERNEL, BLOCK>, reinterpret_cast<const void*>(KERNEL), NAME }

// product kernels
constexpr SmemSpec kSmemDefault{.block = 256, .group = 8, .filter = Filter::Max3, .tail = Tail::Coop,
                                .tail_lanes = 32, .waves = 6, .stats = false, .lockstep = true};
#ifdef RT2_EXPERIMENTS
constexpr SmemSpec kSmemMid{.block = 256, .group = 8, .filter = Filter::Max3, .tail = Tail::Coop, .tail_lanes = 32,
                            .waves = 1, .stats = false};
constexpr SplitSpec kSplitSmall{.waves_per_ray = 4, .group = 8, .filter = Filter::Max3, .waves = 6};
constexpr SmemSpec kSmemFree{.block = 256, .group = 8, .filter = Filter::Max3, .tail = Tail::Coop, .tail_lanes = 32,
                             .waves = 6, .stats = false, .lockstep = false};
constexpr AssistSpec assist12_x(int coop) {
    return AssistSpec{.waves_per_block = 12, .group = 8, .filter = Filter::Max3, .waves = 6, .coop_rays = coop};
}
#endif
constexpr TiledSpec kTiledLarge{.block = 512, .group = 4, .filter = Filter::Max3};
constexpr AssistSpec kAssist12{.waves_per_block = 12, .group = 8, .filter = Filter::Max3, .waves = 6, .coop_rays = 32};
constexpr MfmaSpec kMfmaT8Y4{.block = 256, .waves = 4, .tail_lanes = 8, .imax = true, .minred = true, .ymma = true,
                             .tshift = 12};
// k16 sweep (v_mfma_f32_32x32x16_f16, 8 products per 1,024 pairs)
constexpr MfmaSpec k16_spec(int waves, bool afrag_lds = false, bool diag = false, bool rsplit = false,
                           bool prefetch = false) {
    return MfmaSpec{.block = 256, .waves = waves, .tail_lanes = 8, .imax = true, .prefetch = prefetch,
                    .minred = true, .diag = diag, .ymma = true, .tshift = 12, .k16 = true, .afrag_lds = afrag_lds,
                    .rsplit = rsplit};
}
constexpr MfmaSpec kMfmaK16 = [] {
    MfmaSpec x = k16_spec(3);
    x.lane_lds = true;
    x.serial = 4;
    x.compact = true;
    return x;
}();
constexpr MfmaSpec kMfmaK16W4 = [] {
    MfmaSpec x = kMfmaK16;
    x.waves = 4;
    x.lane_lds = 2;
    return x;
}();
constexpr MfmaSpec kMfmaK5 = [] {
    MfmaSpec x = kMfmaK16;
    x.k5 = true;
    return x;
}();
constexpr MfmaSpec kMfmaK5W4 = [] {
    MfmaSpec x = kMfmaK16W4;
    x.k5 = true;
    return x;
}();
constexpr MfmaSpec kMfmaK5NoTn = [] {
    MfmaSpec x = kMfmaK5;
    x.no_tn = true;
    return x;
}();
constexpr MfmaSpec kMfmaK5NoTnW4 = [] {
    MfmaSpec x = kMfmaK5W4;
    x.no_tn = true;
    return x;
}();
// the small-scene kernel (233) with the cooperative drain at <= 4 live rays
// instead of 8 (config B 189.5 vs 194.4 ms, 1/8 slab 29.0 vs 29.4 ms;
// profiles/r03_coop_ab_configB.json, r03_coop_shard_probe_configB.jsonl)
[[maybe_unused]] constexpr MfmaSpec kMfmaK5NoTnW4C4 = [] {
    MfmaSpec x = kMfmaK5NoTnW4;
    x.tail_lanes = 4;
    return x;
}();
// the 5-product form with workgroup-shared LDS record tiles (rt2_k5_tiles.h):
// 12 waves (3 per SIMD, one workgroup per CU), K = 4 groups per tile
constexpr MfmaSpec k5_tiles_spec(int K, bool no_tn, int tail, bool diag = false) {
    MfmaSpec x = kMfmaK5W4;
    x.block = 768;
    x.waves = 3;
    x.tile_groups = K;
    x.no_tn = no_tn;
    x.tail_lanes = tail;
    x.diag = diag;
    return x;
}
// records resident in LDS (rt2_k5_resident.h): one workgroup per CU (3 or 4
// waves per SIMD), scenes of <= kResGroups 32-triangle groups
constexpr int kResGroups = 38;  // 152 KiB of k5 records (4 KiB per group) of the CU's 160 KiB
constexpr MfmaSpec k5_res_spec(int waves, bool diag = false, int tail = 4) {
    MfmaSpec x = kMfmaK5NoTn;
    x.block = 256 * waves;
    x.waves = waves;
    x.tail_lanes = tail;
    x.lane_lds = 0;
    x.cthr = true;
    x.lockstep = false;
    x.thr_hoist = true;  // the threshold fragment once per sweep (config B 158.9 vs 160.2, 166.3 vs 167.5 ms)
    x.dpp = true;        // the segment's wave maxima by DPP lane moves (159.4 vs 160.4, 163.1 vs 164.6 ms)
    x.res_groups = kResGroups;
    x.diag = diag;
    return x;
}
// the threshold in the K-slots (round 6, MfmaSpec::kthr): the resident kernel on the kt records, schedule `sched`;
// l2: scenes of up to 256 groups, the groups beyond the resident 38 read from L2
constexpr MfmaSpec kt_res_spec(int sched, bool diag = false, bool l2 = false) {
    MfmaSpec x = k5_res_spec(4, diag);
    x.cthr = false;
    x.thr_hoist = false;
    x.kthr = sched;
    x.res_l2 = l2;
    return x;
}
// ... and the LDS-tiled kernel on the kt records (the form of 293), K groups per tile, `waves` per SIMD
constexpr MfmaSpec kt_tiles_spec(int K, int waves, int sched) {
    MfmaSpec x = k5_tiles_spec(K, true, 0);
    x.block = 256 * waves;
    x.waves = waves;
    x.rows80 = true;
    x.lane_lds = 0;
    x.perm_frag = true;
    x.dpp = true;
    x.kthr = sched;
    return x;
}
// the round-6 tiled kernel (above 8,192 triangles): kthr 4, each ray's own W, the tiles streamed with LDS counters
// (MfmaSpec::tile_flow) and issue priority by finishing rank (flow_prio)
constexpr MfmaSpec kt_tiles_flow() {
    MfmaSpec x = kt_tiles_spec(19, 3, 4);
    x.kt_lane_w = true;
    x.tile_flow = true;
    x.flow_prio = true;
    return x;
}
// ... at 4 waves per SIMD (1,024 threads) with the lean lane state (128 VGPRs, 1 spilled): the default
constexpr MfmaSpec kt_tiles_flow4() {
    MfmaSpec x = kt_tiles_flow();
    x.block = 1024;
    x.waves = 4;
    x.lean = true;
    return x;
}
// the round-6 defaults: kthr 4, the lean lane state; l2 = the L2 continuation (39..256 groups), fair = rank slabs
constexpr MfmaSpec kt_res_lean(bool l2, bool fair, bool lane_w = false) {
    MfmaSpec x = kt_res_spec(4, false, l2);
    x.lean = true;
    x.fair_prio = fair;
    x.kt_lane_w = lane_w;
    return x;
}
// the whole-image defaults (353, 355): each ray's own W and issue priority by phase (the exact phase and shading
// above the products: MfmaSpec::phase_prio 4); the rank-slab forms (354, 356) keep fair-share priority instead
constexpr MfmaSpec kt_res_prod(bool l2) {
    MfmaSpec x = kt_res_lean(l2, false, true);
    x.phase_prio = 4;
    return x;
}
constexpr int kResL2Groups = 256;  // render_mfma_k5r with res_l2: 38 groups resident, the rest from L2
constexpr Bvh3Spec kBvhDefault{.block = 256, .thresh = 16, .slab = Slab::Markstein, .waves = 5, .diag = false};

#ifdef RT2_EXPERIMENTS
constexpr SmemSpec smem_x(int g, Filter f, Tail t, int lanes, int w, bool stats = false) {
    return SmemSpec{.block = 256, .group = g, .filter = f, .tail = t, .tail_lanes = lanes, .waves = w, .stats = stats};
}
constexpr SplitSpec split_x(int s, Filter f, int w) {
    return SplitSpec{.waves_per_ray = s, .group = 8, .filter = f, .waves = w};
}
constexpr Bvh3Spec bvh3_x(int t, Slab sl, int w, bool diag = false) {
    return Bvh3Spec{.block = 256, .thresh = t, .slab = sl, .waves = w, .diag = diag};
}
#endif

const Variant kVariants[] = {
    RT2_VARIANT(0, K_SMEM, render_smem<kSmemDefault>, 256, "smem/256/max3f8/coop32/w6/lockstep"),  // default (<= kSmemMaxTris)
    RT2_VARIANT(109, K_BVH4, render_bvh4<kBvhDefault>, 256, "bvh4/256/t16/w5"),           // default (BVH traversal)
    RT2_VARIANT(86, K_TILED, render_tiled<kTiledLarge>, 512, "tiled/512/max3f4"),          // > kSmemMaxTris
    RT2_VARIANT(92, K_ASSIST, render_assist<kAssist12>, 768, "assist12/max3f8/w6"),        // < 4 items per lane
    RT2_VARIANT(136, K_SMEM, render_smem<kSmemDefault>, 256, "smem/256/max3f8/coop32/w6/lockstep"),  // variant 0 forced (id 0 = automatic)
    // default brute-force kernel (DESIGN.md "The 5-product form"): the k16 sweep with U, -V, X from the first K-half,
    // the left-out m.z slots bounded in the threshold; 3 waves per SIMD, and 4 for launches with < 1.5 items per lane
    RT2_VARIANT(227, K_MFMA, render_mfma<kMfmaK5>, 256, "mfma/256/k5/coop8/w3/imax/minred/ymma/t12/llds/ser4/cmp"),
    // scenes of <= 256 groups (8,192 triangles; config B: 38, W: 57, K: 89): the resident kernel (rt2_k5_resident.h:
    // records in LDS for the whole launch, 38 groups, the rest read from L2) with the threshold in the K-slots
    // (MfmaSpec::kthr 4: 8 independent products per group, the two 32-ray blocks interleaved; DESIGN.md "The
    // threshold in the K-slots"), the lean lane state; fair-share issue priority for rank slabs
    RT2_VARIANT(353, K_MFMA, render_mfma_k5r<kt_res_prod(false)>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw/pp4"),
    RT2_VARIANT(354, K_MFMA, render_mfma_k5r<kt_res_lean(false, true, true)>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/fair/dpp/lean/lw"),
    RT2_VARIANT(355, K_MFMA, render_mfma_k5r<kt_res_prod(true)>, 1024, "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/dpp/lean/lw/pp4"),
    RT2_VARIANT(356, K_MFMA, render_mfma_k5r<kt_res_lean(true, true, true)>, 1024, "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/fair/dpp/lean/lw"),
    // the default above 8,192 triangles: the LDS-tiled kernel (rt2_k5_tiles.h; 19-group tiles, fragments in
    // registers) with the threshold in the K-slots, each ray's own W in the bound (round 6; round 5: 293)
    RT2_VARIANT(380, K_MFMA, render_mfma_k5t<kt_tiles_flow4()>, 1024, "mfmat5/1024/kt4/tile19/coop0/w4/cmp/regs/perm/lw/flowp/lean"),
#ifdef RT2_EXPERIMENTS
    // the tile stream at 3 waves per SIMD (380 takes 4 with the lean lane state)
    RT2_VARIANT(370, K_MFMA, render_mfma_k5t<kt_tiles_flow()>, 768, "mfmat5/768/kt4/tile19/coop0/w3/cmp/regs/perm/lw/flowp"),
    // round 6's first tiled default (one workgroup barrier per tile; 370 streams the tiles with LDS counters)
    RT2_VARIANT(351, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_spec(19, 3, 4); x.kt_lane_w = true; return x; }()>, 768, "mfmat5/768/kt4/tile19/coop0/w3/cmp/regs/perm/lw"),
    // round 6's first kthr defaults (the wave's W in the bound; 353-356 take each ray's own)
    RT2_VARIANT(342, K_MFMA, render_mfma_k5r<kt_res_lean(false, false)>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean"),
    RT2_VARIANT(344, K_MFMA, render_mfma_k5r<kt_res_lean(false, true)>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/fair/dpp/lean"),
    RT2_VARIANT(345, K_MFMA, render_mfma_k5r<kt_res_lean(true, false)>, 1024, "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/dpp/lean"),
    RT2_VARIANT(346, K_MFMA, render_mfma_k5r<kt_res_lean(true, true)>, 1024, "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/fair/dpp/lean"),
    // the defaults of rounds 4-5 (round 6 replaced them by the kthr resident kernels 353-356 and the kthr tiles 351)
    RT2_VARIANT(293, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = k5_tiles_spec(19, true, 0); x.rows80 = true; x.lane_lds = 0; x.cthr = true; x.perm_frag = true; return x; }()>, 768, "mfmat5/768/k5/notn/tile19/coop0/w3/cmp/regs/cthr/perm"),
    // (round 4) scenes of <= 8,192 triangles (records L2-resident): the same without the -tn term (4 products per block) and
    // with the threshold in the products' accumulator (MfmaSpec::cthr, DESIGN.md "The threshold in the
    // accumulator"), 4 waves (packed path state, Y fragments read per block: 263), or 3 when the packed fields do not
    // hold the image / rays / bounces (262)
    RT2_VARIANT(263, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5NoTnW4C4; x.cthr = true; x.ylds = 1; return x; }()>, 256, "mfma/256/k5/notn/coop4/w4/imax/minred/ymma/t12/llds2/ser4/cmp/cthr/yl1"),
    RT2_VARIANT(262, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5NoTn; x.cthr = true; return x; }()>, 256, "mfma/256/k5/notn/coop8/w3/imax/minred/ymma/t12/llds/ser4/cmp/cthr"),
    // LDS record tiles shared by the workgroup (rt2_k5_tiles.h; DESIGN.md "LDS record tiles"), the default above
    // 8,192 triangles: 10-group tiles, path state in registers, the threshold in the accumulator
    RT2_VARIANT(217, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = k5_tiles_spec(10, true, 0); x.rows80 = true; x.lane_lds = 0; x.cthr = true; return x; }()>, 768, "mfmat5/768/k5/notn/tile10/coop0/w3/cmp/rows80/regs/cthr"),
    // scenes of <= 38 groups (1,216 triangles: config B): every group's records resident in LDS for the whole
    // launch (rt2_k5_resident.h), fragments built in registers by v_permlane32_swap, waves run free
    RT2_VARIANT(282, K_MFMA, render_mfma_k5r<k5_res_spec(4)>, 1024, "mfmar/1024/k5/notn/res38/coop4/w4/cmp/cthr/dpp"),
    // ... with fair-share issue priority (rank slabs: < kResSlabItems items per lane; DESIGN.md "Fair-share issue
    // priority")
    RT2_VARIANT(298, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = k5_res_spec(4); x.fair_prio = true; return x; }()>, 1024, "mfmar/1024/k5/notn/res38/coop4/w4/cmp/cthr/fair/dpp"),
    // records resident in LDS at 3 waves per SIMD; the resident kernel's diagnostic counters
    RT2_VARIANT(280, K_MFMA, render_mfma_k5r<k5_res_spec(3)>, 768, "mfmar/768/k5/notn/res38/coop4/w3/cmp/cthr/dpp"),
    RT2_VARIANT(287, K_MFMA, render_mfma_k5r<k5_res_spec(4, true)>, 1024, "mfmar/1024/k5/notn/res38/coop4/w4/cmp/cthr/diag/dpp"),
    // the threshold in the K-slots (round 6): schedules 1 (four products, then the reduction) / 2 (cthr's order) /
    // 3 (no fences); fair-share priority; diagnostic counters; the L2 continuation for 39..256 groups
    RT2_VARIANT(320, K_MFMA, render_mfma_k5r<kt_res_spec(1)>, 1024, "mfmar/1024/kt1/res38/coop4/w4/cmp/dpp"),
    RT2_VARIANT(321, K_MFMA, render_mfma_k5r<kt_res_spec(2)>, 1024, "mfmar/1024/kt2/res38/coop4/w4/cmp/dpp"),
    RT2_VARIANT(322, K_MFMA, render_mfma_k5r<kt_res_spec(3)>, 1024, "mfmar/1024/kt3/res38/coop4/w4/cmp/dpp"),
    RT2_VARIANT(323, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(1); x.fair_prio = true; return x; }()>, 1024, "mfmar/1024/kt1/res38/coop4/w4/cmp/fair/dpp"),
    RT2_VARIANT(324, K_MFMA, render_mfma_k5r<kt_res_spec(1, true)>, 1024, "mfmar/1024/kt1/res38/coop4/w4/cmp/diag/dpp"),
    RT2_VARIANT(325, K_MFMA, render_mfma_k5r<kt_res_spec(1, false, true)>, 1024, "mfmarl2/1024/kt1/res38l2/coop4/w4/cmp/dpp"),
    // ... at 3 waves per SIMD (168 VGPRs: the four products before the reduction fit), with the next group's
    // operands read ahead
    RT2_VARIANT(326, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(1); x.block = 768; x.waves = 3; return x; }()>, 768, "mfmar/768/kt1/res38/coop4/w3/cmp/dpp"),
    RT2_VARIANT(327, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(1); x.block = 768; x.waves = 3; x.prefetch = true; return x; }()>, 768, "mfmar/768/kt1/res38/coop4/w3/cmp/dpp/pf"),
    RT2_VARIANT(328, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(1); x.prefetch = true; return x; }()>, 1024, "mfmar/1024/kt1/res38/coop4/w4/cmp/dpp/pf"),
    // ... schedule 4: the two 32-ray blocks interleaved (each wave's products beside its own reduction)
    RT2_VARIANT(329, K_MFMA, render_mfma_k5r<kt_res_spec(4)>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp"),
    RT2_VARIANT(336, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(4); x.fair_prio = true; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/fair/dpp"),
    RT2_VARIANT(337, K_MFMA, render_mfma_k5r<kt_res_spec(4, false, true)>, 1024, "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/dpp"),
    RT2_VARIANT(338, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(4, false, true); x.fair_prio = true; return x; }()>, 1024, "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/fair/dpp"),
    RT2_VARIANT(339, K_MFMA, render_mfma_k5r<kt_res_spec(4, true)>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/diag/dpp"),
    // ... the fold as two chains (kthr 5); speed-of-light probe without the exact phase (WRONG images: A/B with
    // --no-check)
    RT2_VARIANT(340, K_MFMA, render_mfma_k5r<kt_res_spec(5)>, 1024, "mfmar/1024/kt5/res38/coop4/w4/cmp/dpp"),
    RT2_VARIANT(341, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(4); x.sol = 2; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/sol2"),
    // ... with the lean lane state (x, y from the item, segments counted per wave)
    RT2_VARIANT(342, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(4); x.lean = true; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean"),
    RT2_VARIANT(343, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(5); x.lean = true; return x; }()>, 1024, "mfmar/1024/kt5/res38/coop4/w4/cmp/dpp/lean"),
    // ... the exact phase with the next triangle requested ahead (vector loads)
    RT2_VARIANT(347, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_lean(false, false); x.exact_pf = true; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/xpf"),
    // ... W per ray (kt_lane_w: a tighter threshold, fewer exact tests)
    RT2_VARIANT(348, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_lean(false, false); x.kt_lane_w = true; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw"),
    RT2_VARIANT(349, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_lean(false, false); x.kt_lane_w = true; x.exact_pf = true; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw/xpf"),
    RT2_VARIANT(350, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_spec(4, true); x.lean = true; x.kt_lane_w = true; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/diag/dpp/lean/lw"),
    // ... on the LDS-tiled kernel (the form of 293): 19-group tiles at 3 waves per SIMD (schedules 1, 2), 16-group
    // tiles at 4 waves
    RT2_VARIANT(330, K_MFMA, render_mfma_k5t<kt_tiles_spec(19, 3, 1)>, 768, "mfmat5/768/kt1/tile19/coop0/w3/cmp/regs/perm"),
    RT2_VARIANT(331, K_MFMA, render_mfma_k5t<kt_tiles_spec(19, 3, 2)>, 768, "mfmat5/768/kt2/tile19/coop0/w3/cmp/regs/perm"),
    RT2_VARIANT(332, K_MFMA, render_mfma_k5t<kt_tiles_spec(19, 3, 4)>, 768, "mfmat5/768/kt4/tile19/coop0/w3/cmp/regs/perm"),
    RT2_VARIANT(333, K_MFMA, render_mfma_k5t<kt_tiles_spec(16, 4, 1)>, 1024, "mfmat5/1024/kt1/tile16/coop0/w4/cmp/regs/perm"),
    RT2_VARIANT(335, K_MFMA, render_mfma_k5t<kt_tiles_spec(16, 4, 4)>, 1024, "mfmat5/1024/kt4/tile16/coop0/w4/cmp/regs/perm"),
    // ... the tiles as a stream with LDS counters (MfmaSpec::tile_flow): with its diagnostic clocks; without flow_prio
    RT2_VARIANT(368, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_flow(); x.diag = true; return x; }()>, 768, "mfmat5/768/kt4/tile19/coop0/w3/cmp/regs/perm/lw/flowp/diag"),
    RT2_VARIANT(369, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_flow(); x.flow_prio = false; return x; }()>, 768, "mfmat5/768/kt4/tile19/coop0/w3/cmp/regs/perm/lw/flow"),
    // ... 4 waves per SIMD with 16-group tiles; the lean lane state at 3 waves
    RT2_VARIANT(381, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_flow4(); x.tile_groups = 16; return x; }()>, 1024, "mfmat5/1024/kt4/tile16/coop0/w4/cmp/regs/perm/lw/flowp/lean"),
    RT2_VARIANT(382, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_flow(); x.lean = true; return x; }()>, 768, "mfmat5/768/kt4/tile19/coop0/w3/cmp/regs/perm/lw/flowp/lean"),
    RT2_VARIANT(385, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_flow4(); x.flow_prio = false; return x; }()>, 1024, "mfmat5/1024/kt4/tile19/coop0/w4/cmp/regs/perm/lw/flow/lean"),
    RT2_VARIANT(386, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_flow4(); x.tail_lanes = 4; return x; }()>, 1024, "mfmat5/1024/kt4/tile19/coop4/w4/cmp/regs/perm/lw/flowp/lean"),
    // ... issue priority by phase (MfmaSpec::phase_prio 1 / 2 / 3; 353 takes 4); 391 = 353 without it
    RT2_VARIANT(387, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_lean(false, false, true); x.phase_prio = 1; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw/pp1"),
    RT2_VARIANT(388, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_lean(false, false, true); x.phase_prio = 2; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw/pp2"),
    RT2_VARIANT(389, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = kt_res_lean(false, false, true); x.phase_prio = 3; return x; }()>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw/pp3"),
    RT2_VARIANT(391, K_MFMA, render_mfma_k5r<kt_res_lean(false, false, true)>, 1024, "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw"),
    RT2_VARIANT(352, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_spec(19, 3, 1); x.kt_lane_w = true; return x; }()>, 768, "mfmat5/768/kt1/tile19/coop0/w3/cmp/regs/perm/lw"),
    RT2_VARIANT(334, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = kt_tiles_spec(19, 3, 1); x.diag = true; return x; }()>, 768, "mfmat5/768/kt1/tile19/coop0/w3/cmp/regs/perm/diag"),
    RT2_VARIANT(299, K_MFMA, render_mfma_k5r<[] { MfmaSpec x = k5_res_spec(4, true); x.fair_prio = true; return x; }()>, 1024, "mfmar/1024/k5/notn/res38/coop4/w4/cmp/cthr/fair/diag/dpp"),
    // earlier choices of rounds 3-4 (the 5-product form before and after the threshold moved into the accumulator,
    // the first tile forms), kept for A/B; rounds 2-3's 16x16x32 and k16 kernels are in git history
    RT2_VARIANT(231, K_MFMA, render_mfma<kMfmaK5NoTn>, 256, "mfma/256/k5/notn/coop8/w3/imax/minred/ymma/t12/llds/ser4/cmp"),
    RT2_VARIANT(243, K_MFMA, render_mfma<kMfmaK5NoTnW4C4>, 256, "mfma/256/k5/notn/coop4/w4/imax/minred/ymma/t12/llds2/ser4/cmp"),
    RT2_VARIANT(213, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = k5_tiles_spec(10, true, 0); x.rows80 = true; x.lane_lds = 0; return x; }()>, 768, "mfmat5/768/k5/notn/tile10/coop0/w3/cmp/rows80/regs"),
    RT2_VARIANT(252, K_MFMA, render_mfma_k5t<k5_tiles_spec(4, true, 0)>, 768, "mfmat5/768/k5/notn/tile4/coop0/w3/llds2/cmp"),
    RT2_VARIANT(228, K_MFMA, render_mfma<kMfmaK5W4>, 256, "mfma/256/k5/coop8/w4/imax/minred/ymma/t12/llds2/ser4/cmp"),
    RT2_VARIANT(233, K_MFMA, render_mfma<kMfmaK5NoTnW4>, 256, "mfma/256/k5/notn/coop8/w4/imax/minred/ymma/t12/llds2/ser4/cmp"),
    RT2_VARIANT(250, K_MFMA, render_mfma_k5t<k5_tiles_spec(4, false, 0)>, 768, "mfmat5/768/k5/tile4/coop0/w3/llds2/cmp"),
    RT2_VARIANT(260, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5NoTnW4C4; x.cthr = true; return x; }()>, 256, "mfma/256/k5/notn/coop4/w4/imax/minred/ymma/t12/llds2/ser4/cmp/cthr"),
    RT2_VARIANT(261, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5NoTnW4C4; x.cthr = true; x.ylds = 2; return x; }()>, 256, "mfma/256/k5/notn/coop4/w4/imax/minred/ymma/t12/llds2/ser4/cmp/cthr/ylds"),
    RT2_VARIANT(212, K_MFMA, render_mfma_k5t<[] { MfmaSpec x = k5_tiles_spec(8, true, 0); x.rows80 = true; x.lane_lds = 0; return x; }()>, 768, "mfmat5/768/k5/notn/tile8/coop0/w3/cmp/rows80/regs"),
    RT2_VARIANT(246, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5NoTnW4C4; x.rows80 = true; return x; }()>, 256, "mfma/256/k5/notn/coop4/w4/imax/minred/ymma/t12/llds2/ser4/cmp/rows80"),
    RT2_VARIANT(251, K_MFMA, render_mfma_k5t<k5_tiles_spec(4, false, 0, true)>, 768, "mfmat5/768/k5/tile4/coop0/w3/llds2/cmp/diag"),
    // diagnostic builds (group / survivor / exact-test counters, wave timeline)
    RT2_VARIANT(239, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5NoTnW4; x.diag = true; return x; }()>, 256, "mfma/256/k5/notn/coop8/w4/imax/minred/ymma/t12/llds2/ser4/cmp/diag"),
    RT2_VARIANT(232, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5NoTn; x.diag = true; return x; }()>, 256, "mfma/256/k5/notn/coop8/w3/imax/minred/ymma/t12/llds/ser4/cmp/diag"),
    RT2_VARIANT(229, K_MFMA, render_mfma<[] { MfmaSpec x = kMfmaK5; x.diag = true; return x; }()>, 256, "mfma/256/k5/coop8/w3/imax/minred/ymma/t12/llds/ser4/cmp/diag"),
    // scalar-path and BVH kernels of rounds 1-2 (DESIGN.md "Tried and measured"; parity-tested in the experiment build)
    RT2_VARIANT(67, K_SMEM, render_smem<kSmemMid>, 256, "smem/256/max3f8/coop32"),         // round-1 choice, 1-4 items per lane
    RT2_VARIANT(85, K_SPLIT, render_split<kSplitSmall>, 256, "split4/max3f8/w6"),          // round-1 choice, < 1 item per lane
    RT2_VARIANT(53, K_BVH3, render_bvh3<kBvhDefault>, 256, "bvh3/256/t16/w5"),            // round-1/2 BVH default
    RT2_VARIANT(106, K_SMEM, render_smem<kSmemFree>, 256, "smem/256/max3f8/coop32/w6/free"),  // round-1 default
    RT2_VARIANT(37, K_BVH, render_bvh<BvhSpec{256}>, 256, "bvh/256"),
    RT2_VARIANT(40, K_BVH2, (render_bvh2<Bvh2Spec{256, 16}>), 256, "bvh2/256/t16"),
    RT2_VARIANT(41, K_BVH2, (render_bvh2<Bvh2Spec{256, 8}>), 256, "bvh2/256/t8"),
    RT2_VARIANT(43, K_BVH2, (render_bvh2<Bvh2Spec{128, 16}>), 128, "bvh2/128/t16"),
    RT2_VARIANT(45, K_BVH2, (render_bvh2<Bvh2Spec{256, 1}>), 256, "bvh2/256/t1"),
    RT2_VARIANT(46, K_BVH3, render_bvh3<bvh3_x(16, Slab::Markstein, 1)>, 256, "bvh3/256/t16"),
    RT2_VARIANT(47, K_BVH3, render_bvh3<bvh3_x(8, Slab::Markstein, 1)>, 256, "bvh3/256/t8"),
    RT2_VARIANT(48, K_BVH3, render_bvh3<bvh3_x(24, Slab::Markstein, 1)>, 256, "bvh3/256/t24"),
    RT2_VARIANT(50, K_BVH3, render_bvh3<bvh3_x(16, Slab::Binary64, 1)>, 256, "bvh3/256/t16/div64"),
    RT2_VARIANT(54, K_BVH3, render_bvh3<bvh3_x(8, Slab::Markstein, 5)>, 256, "bvh3/256/t8/w5"),
    RT2_VARIANT(55, K_BVH3, render_bvh3<bvh3_x(16, Slab::Filtered, 5)>, 256, "bvh3/256/t16/filt/w5"),
    RT2_VARIANT(58, K_BVH3, render_bvh3<bvh3_x(16, Slab::Markstein, 5, true)>, 256, "bvh3/256/t16/w5/DIAG"),
    RT2_VARIANT(64, K_SMEM, render_smem<smem_x(8, Filter::Five, Tail::Team, 32, 1)>, 256, "smem/256/masked8/team32"),
    RT2_VARIANT(66, K_SMEM, render_smem<smem_x(8, Filter::Five, Tail::Team, 64, 1)>, 256, "smem/256/masked8/team64"),
    RT2_VARIANT(74, K_SMEM, render_smem<smem_x(4, Filter::Plk, Tail::Coop, 32, 1)>, 256, "smem/256/plk4/coop32"),
    RT2_VARIANT(76, K_SMEM, render_smem<smem_x(8, Filter::Plk, Tail::Coop, 32, 1)>, 256, "smem/256/plk8/coop32"),
    RT2_VARIANT(79, K_SMEM, render_smem<smem_x(8, Filter::Plk, Tail::Coop, 32, 6)>, 256, "smem/256/plk8/coop32/w6"),
    RT2_VARIANT(80, K_SMEM, render_smem<smem_x(2, Filter::Plk, Tail::Coop, 32, 1)>, 256, "smem/256/plk2/coop32"),
    RT2_VARIANT(82, K_SMEM, render_smem<smem_x(8, Filter::Max3, Tail::Coop, 32, 1, true)>, 256,
                "smem/256/max3f8/coop32/STATS"),
#endif
};
constexpr size_t kResidentMaxBytes = 112 * 1024;
constexpr int kSmemMaxTris = 131072;  // scalar path up to 6.3 MB of records (config C: 781 vs 817 ms tiled; config E: tiled 1,704 vs 2,312 ms)
constexpr int kDefaultBrute = 0;
constexpr int kDefaultBvh = 109;
constexpr int kLargeScene = 86;  // tiled/512/max3f4: LDS tiles above kSmemMaxTris triangles
constexpr int kSlab = 92;        // assist12/max3f8/w6: fewer than 4 items per lane (multi-GPU slabs)
constexpr int kMfmaSlabMaxTris = 8192;  // = kResL2Groups x 32: the resident kernel with its L2 continuation
constexpr int kMfmaRes = 353;      // <= kResGroups groups (config B): every record resident in LDS, 4 waves per SIMD,
                                   // the threshold in the K-slots (kthr 4, each ray's own W in the bound), the lean
                                   // lane state (rt2_k5_resident.h; DESIGN.md "The threshold in the K-slots"): config
                                   // B 149.0 vs 152.8 ms (342, the wave's W) vs 154.2-165.3 ms for round 5's 282 in
                                   // A/Bs, identical images
constexpr int kMfmaResSlab = 354;  // ... launches with < kResSlabItems items per resident lane (rank slabs): the
                                   // same kernel with fair-share issue priority (MfmaSpec::fair_prio; round 5: 298)
constexpr unsigned long long kResSlabItems = 6;
constexpr int kMfmaResL2 = 355;    // 39..256 groups (configs W, K): 38 groups resident, the rest read from L2
                                   // (MfmaSpec::res_l2): config W 28.7 vs 46.5 ms, K 306.8 vs 362.1 ms for round 4-5's
                                   // L2-resident 263 (A/B of the wave-W form 337, identical images)
constexpr int kMfmaResL2Slab = 356;  // ... its rank slabs (fair-share priority)
constexpr int kMfmaTiles = 380;    // larger scenes: the LDS-tiled kernel (rt2_k5_tiles.h: one 16-wave workgroup per
                                   // CU, 19-group record tiles, fragments in registers) with the threshold in the
                                   // K-slots and each ray's own W (config C sample 962 vs 1,076 ms, config E sample
                                   // 1,081 vs 1,230 ms for round 5's 293), the tiles streamed with LDS counters and
                                   // rank priority (full-width config C frame 5,268 vs 5,369 ms, config E 5,447 vs
                                   // 5,522 ms for 351), 4 waves per SIMD with the lean lane state (C frame 5,037 vs
                                   // 5,237 ms, E 5,285 vs 5,451 ms for 370; A/B, identical images)
constexpr int kMfma = 227;  // mfma/.../k5/...: the matrix-core filter on v_mfma_f32_32x32x16_f16, 5 products per
                            // 32-ray block (DESIGN.md "The 5-product form"), registers only; larger scenes whose
                            // packed path state cannot hold the launch

constexpr bool is_bvh(int kind) { return kind >= K_BVH && kind <= K_BVH4; }

const Variant* find_variant(int id) {
    for (const Variant& v : kVariants)
        if (v.id == id) return &v;
    return nullptr;
}
hipError_t variant_occupancy(const Variant& v, int* occ, size_t lds) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, v.kernel, v.block, lds);
}
}  // namespace

extern "C" int rt2_scene_set_variant(rt2_scene* s, int variant) {
    if (!s) {
        rt2h::set_error("rt2_scene_set_variant: null scene");
        return -1;
    }
    if (variant != 0 && !find_variant(variant)) {
        rt2h::set_error("rt2_scene_set_variant: variant " + std::to_string(variant) +
                        " is not in this build (experiment variants need make EXPERIMENTS=1)");
        return -1;
    }
    s->variant = variant;
    return variant;
}

extern "C" const char* rt2_variant_name(int v) {
    const Variant* V = find_variant(v);
    return V ? V->name : nullptr;
}

// Not in rt2.h (diagnostics): the occupancy API's blocks per CU and the
// kernel's register counts (hipFuncGetAttributes) for variant v.
extern "C" int rt2_variant_occupancy(int v, int* api_blocks, int* num_regs, int* local_bytes) {
    const Variant* V = find_variant(v);
    if (!V) return -1;
    int occ = 0;
    HIPCHECK(variant_occupancy(*V, &occ, 0));
    hipFuncAttributes a;
    HIPCHECK(hipFuncGetAttributes(&a, V->kernel));
    if (api_blocks) *api_blocks = occ;
    if (num_regs) *num_regs = a.numRegs;
    if (local_bytes) *local_bytes = (int)a.localSizeBytes;
    return 0;
}

extern "C" int rt2_render(rt2_scene* s, const rt2_uniforms* u, uint32_t frame_begin, uint32_t frame_count,
                          rt2_shard sh, float* d_accum, uint32_t* d_accum8, void* stream) {
    if (!s || !u || !d_accum) {
        rt2h::set_error("rt2_render: null argument");
        return -1;
    }
    if ((!u->basicShading && u->numRaysPerPixel < 1) || u->width < 1 || u->height < 1) {
        rt2h::set_error("rt2_render: numRaysPerPixel, width and height must be >= 1");
        return -1;
    }
    const int rows = rt2_shard_rows((int)u->height, sh);
    if (rows < 0) {
        rt2h::set_error("rt2_render: bad shard");
        return -1;
    }
    if (frame_count == 0 || rows == 0) return 0;
    // frame-major items keep one colour plane per frame: beyond frame_scratch_cap
    // of planes (or 2^32 items), render consecutive frame chunks — the
    // accumulation stays in frame order, so the sums are unchanged
    if (!u->basicShading && s->split_frames && frame_count > 1) {
        const unsigned long long npix = (unsigned long long)rows * u->width;
        unsigned long long chunk = std::max<unsigned long long>(1, s->frame_scratch_cap / (npix * sizeof(float4)));
        chunk = std::min<unsigned long long>(chunk, 0xfffffffeull / std::max<unsigned long long>(npix, 1));
        if (chunk < frame_count) {
            for (unsigned long long f0 = 0; f0 < frame_count; f0 += chunk) {
                const uint32_t fc = (uint32_t)std::min<unsigned long long>(chunk, frame_count - f0);
                const int rc = rt2_render(s, u, frame_begin + (uint32_t)f0, fc, sh, d_accum, d_accum8, stream);
                if (rc != 0) return rc;
            }
            return 0;
        }
    }
    HIPCHECK(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;

    RenderParams p;
    std::memset(&p, 0, sizeof(p));
    p.tri = s->d_tri;
    p.plk = s->plk_ok ? s->d_plk : nullptr;
    p.plk_A = s->plk_A;
    p.mfma_frag = s->d_mfma;
    p.mfma_tau = s->d_mfma_tau;
    p.mfma_A = s->mfma_A;
    p.mfma_k16_frag = s->d_mfma_k16;
    p.mfma_k16_tau = s->d_mfma_k16_tau;
    p.mfma_k16_bnd = s->d_mfma_k16_bnd;
    p.mfma_kt_frag = s->d_mfma_kt;
    p.tri_mtl = s->d_mtl;
    p.raw = s->d_raw;
    p.texels = s->d_texels;
    p.tex_desc = s->d_tex_desc;
    p.n_tex = s->n_tex;
    p.num_textures = u->numTextures;
    p.mats = s->d_mats;
    p.n_tris = s->n_tris;
    p.n_mats = s->n_mats;
    p.W = (int)u->width;
    p.H = (int)u->height;
    p.maxBounce = u->maxBounceCount;
    p.R = u->numRaysPerPixel;
    p.envLight = u->environmentalLight;
    auto cp = [](float* d, const rt2_vec4& v) {
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
    };
    cp(p.cam, u->cameraPos);
    cp(p.vpRight, u->viewportRight);
    cp(p.vpUp, u->viewportUp);
    cp(p.vpFront, u->viewportFront);
    cp(p.pixR, u->pixelRight);
    cp(p.pixU, u->pixelUp);
    cp(p.defR, u->defocusDiskRight);
    cp(p.defU, u->defocusDiskUp);
    p.frame_begin = frame_begin;
    p.frame_count = frame_count;
    p.tile_rows = sh.tile_rows;
    p.rank = sh.rank;
    p.nranks = sh.nranks;
    p.n_pix = (unsigned long long)rows * (unsigned long long)p.W;
    p.n_items = p.n_pix;
    if (p.n_pix >= 0xffffffffull) {
        rt2h::set_error("rt2_render: more than 2^32-1 pixels in one shard");
        return -1;
    }
    p.accum = reinterpret_cast<float4*>(d_accum);
    p.accum8 = reinterpret_cast<uint4*>(d_accum8);
    p.item_counter = s->d_counters;
    p.seg_counter = s->d_counters + 1;
    p.tile_tris = kTileTris;
    p.wave_log = s->wave_log;
    p.wave_log_n = s->wave_log_n;

    // renders of one scene share its counters and scratch (frame planes, cost
    // map, pixel order): a render waits for the scene's previous one, whatever
    // stream that was issued on
    if (s->last_launch_valid) HIPCHECK(hipStreamWaitEvent(st, s->last_launch, 0));
    HIPCHECK(hipMemsetAsync(s->d_counters, 0, sizeof(unsigned long long), st));
    // items in 8 contiguous regions, one per group of workgroups sharing an
    // XCD's L2 (blockIdx % 8): neighbouring pixels' rays walk the same BVH
    // lines in one L2 (config C BVH: 2,701 vs 2,783 ms; brute force ±0)
    if (!s->d_region_ctr) HIPCHECK(hipMalloc(&s->d_region_ctr, 8 * 128));
    HIPCHECK(hipMemsetAsync(s->d_region_ctr, 0, 8 * 128, st));
    p.region_ctr = s->d_region_ctr;
    HIPCHECK(hipMemsetAsync(s->d_counters + 6, 0xff, sizeof(unsigned long long), st));  // diag: min wave end
    HIPCHECK(hipMemsetAsync(s->d_counters + 7, 0, sizeof(unsigned long long), st));     // diag: max wave end
    p.nodes = s->d_nodes;
    p.stack_slots = s->bvh_depth + 2;
    if (u->basicShading) {  // traceBasic preview: one thread per pixel
        p.basicShadow = u->basicShadingShadow;
        cp(p.light, u->basicShadingLightPosition);
        constexpr int kBasicBlock = 256;
        const unsigned long long blocks = (p.n_items + kBasicBlock - 1) / kBasicBlock;
        if (s->traversal == RT2_TRAVERSAL_BVH) {
            const size_t lds = (size_t)p.stack_slots * kBasicBlock * sizeof(int);
            hipLaunchKernelGGL((render_basic<kBasicBlock, true>), dim3((unsigned)blocks), dim3(kBasicBlock), lds, st,
                               p);
            s->last_kind = K_BVH;
        } else {
            hipLaunchKernelGGL((render_basic<kBasicBlock, false>), dim3((unsigned)blocks), dim3(kBasicBlock), 0, st,
                               p);
            s->last_kind = K_SMEM;
        }
        HIPCHECK(hipGetLastError());
        if (!s->last_launch) HIPCHECK(hipEventCreateWithFlags(&s->last_launch, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(s->last_launch, st));
        s->last_launch_valid = true;
        s->last_variant = -1;
        s->samples += p.n_items * (unsigned long long)frame_count;
        s->tests_per_seg = (unsigned long long)s->n_tris;
        return 0;
    }
    // several frames: frame-major (frame, pixel) items into a scratch buffer,
    // then frame_accumulate (finer work items: a shorter tail)
    if (frame_count > 1 && s->split_frames && p.n_pix * frame_count < 0xffffffffull) {
        const size_t need = (size_t)p.n_pix * frame_count * sizeof(float4);
        if (need > s->fb_bytes) {
            if (s->d_fb) HIPCHECK(hipFree(s->d_fb));
            s->d_fb = nullptr;
            s->fb_bytes = 0;
            HIPCHECK(hipMalloc(&s->d_fb, need));
            s->fb_bytes = need;
        }
        p.frame_split = 1;
        p.frame_buf = s->d_fb;
        p.n_items = p.n_pix * frame_count;
    }
    // cost-ordered items: the previous launch's per-pixel costs (same slab)
    // give this launch's pixel order, most expensive first (a shorter tail)
    if (s->cost_order) {
        if (s->cost_cap < p.n_pix) {
            (void)hipFree(s->d_cost);
            (void)hipFree(s->d_order);
            s->d_cost = s->d_order = nullptr;
            s->cost_cap = 0;
            s->cost_npix = 0;
            HIPCHECK(hipMalloc(&s->d_cost, p.n_pix * sizeof(uint32_t)));
            HIPCHECK(hipMalloc(&s->d_order, p.n_pix * sizeof(uint32_t)));
            if (!s->d_hist) HIPCHECK(hipMalloc(&s->d_hist, 32 * sizeof(uint32_t)));
            s->cost_cap = p.n_pix;
        }
        const int key[4] = {(int)u->width, sh.tile_rows, sh.rank, sh.nranks};
        const bool valid = s->cost_npix == p.n_pix && std::memcmp(key, s->cost_key, sizeof(key)) == 0;
        const unsigned long long runs = p.n_pix / 64;
        if (valid && runs > 0) {
            const unsigned blocks = (unsigned)std::min<unsigned long long>((runs + 255) / 256, 2048);
            HIPCHECK(hipMemsetAsync(s->d_hist, 0, 32 * sizeof(uint32_t), st));
            hipLaunchKernelGGL(cost_histogram, dim3(blocks), dim3(256), 0, st, s->d_cost, runs, s->d_hist);
            hipLaunchKernelGGL(cost_offsets, dim3(1), dim3(64), 0, st, s->d_hist);
            hipLaunchKernelGGL(cost_scatter, dim3(blocks), dim3(256), 0, st, s->d_cost, runs, s->d_hist, s->d_order);
            HIPCHECK(hipGetLastError());
            p.order = s->d_order;
            p.n_runs = (uint32_t)runs;
        }
        // the cost map keeps each item's start clock in the pixel's own slot:
        // with frame-major items several frames of one pixel run at once, so
        // only frame 0's item of each pixel measures (one
        // writer per slot; a frame-split launch's map is its frame 0's cost)
        p.cost_out = s->d_cost;
        s->cost_npix = p.n_pix;
        std::memcpy(s->cost_key, key, sizeof(key));
    }
    const size_t resident_bytes = (size_t)3 * sizeof(float4) * (size_t)std::max(s->n_tris, 1);
    const bool fits = resident_bytes <= kResidentMaxBytes;
    // explicit variant (rt2_scene_set_variant) when it exists in this build and
    // matches the traversal; otherwise the automatic choice: the matrix-core
    // filter kernel for small scenes (config B: 1,208 triangles; the
    // scalar-path kernel when the scene is outside its range), LDS-tiled sweep
    // for large ones (config E: 1M triangles)
    const Variant* VP = s->variant > 0 ? find_variant(s->variant) : nullptr;
    if (VP && ((s->traversal == RT2_TRAVERSAL_BVH) != is_bvh(VP->kind))) VP = nullptr;
    if (VP && VP->kind == K_RESIDENT && !fits) VP = nullptr;  // cannot hold this scene
    const bool res_fits = (s->n_tris + 31) / 32 <= kResGroups;  // render_mfma_k5r's LDS holds every record group
    if (VP && !res_fits && std::strncmp(VP->name, "mfmar/", 6) == 0) VP = nullptr;
    if (VP && (s->n_tris + 31) / 32 > kResL2Groups && std::strncmp(VP->name, "mfmarl2/", 8) == 0) VP = nullptr;
    if (VP && (VP->kind == K_MFMA || VP->kind == K_MASSIST) && !s->mfma_ok) VP = nullptr;  // scene outside the filter's range
    // the packed path state (lane_lds = 2) holds 16-bit x, y, rays per pixel and 12-bit bounce counts
    const bool packed = u->width <= 65535 && u->height <= 65535 && u->maxBounceCount <= 4095 &&
                        u->numRaysPerPixel <= 65535;
    if (VP && !packed && std::strstr(VP->name, "llds2")) VP = nullptr;
    if (!VP && s->traversal == RT2_TRAVERSAL_BVH) VP = find_variant(kDefaultBvh);
    if (!VP) {
        int vi = s->n_tris <= kSmemMaxTris ? kDefaultBrute : kLargeScene;
        if (s->mfma_ok && find_variant(kMfma)) {
            // the filter on the matrix cores (rt2_mfma.h) for whole images and
            // rank slabs alike (its compaction of <= 32 live rays serves the
            // slabs' tails) and every scene size: config E's 1M triangles too
            // (3.9 vs 6.9 s for kLargeScene on a 480x270 sample)
            vi = kMfma;
            // Scenes of up to 256 groups: the resident kernel (its path state
            // in registers: no packed-field limits).  Larger scenes stream
            // their records from the MALL unless the workgroup shares them:
            // the LDS-tiled kernel (one 12-wave workgroup per CU), without the
            // -tn term (config C 26.94 vs 29.19 s with it; config E sample
            // 1.56 vs 1.60 s); its path state stays in registers too
            if (s->n_tris <= kMfmaSlabMaxTris) {
                // the resident kernel: every group resident in LDS (<= 38) or
                // the first 38 resident and the rest read from L2 (<= 256);
                // a SIMD's waves start together with a few items per lane:
                // fair share, so that they also end together (DESIGN.md
                // "Fair-share issue priority")
                const unsigned long long lanes = (unsigned long long)s->num_cus * (unsigned long long)find_variant(kMfmaRes)->block;
                const bool slab = p.n_items < kResSlabItems * lanes;
                vi = res_fits ? (slab ? kMfmaResSlab : kMfmaRes) : (slab ? kMfmaResL2Slab : kMfmaResL2);
            } else if (find_variant(kMfmaTiles)) {
                vi = kMfmaTiles;
            }
        } else if (vi == kDefaultBrute) {
            // scenes outside the matrix filter's range (mfma_ok = 0):
            // items per resident lane decide the tail: a lane ends on a whole
            // item (a pixel-frame's rays share one RNG stream), so with few
            // items per lane the last round runs partly empty.  At >= 4 per
            // lane (a full config B image) the 6-wave scalar-path kernel; below
            // (the 1/2, 1/4, 1/8 slabs of config B on 2, 4, 8 GPUs) the assist
            // kernel, whose idle waves sweep triangle chunks of the busy
            // waves' rays
            const Variant* W = find_variant(kSlab);
            int occ0 = 0;
            HIPCHECK(variant_occupancy(*W, &occ0, 0));
            const unsigned long long lanes = (unsigned long long)s->num_cus * (unsigned long long)std::max(occ0, 1) * W->block;
            if (p.n_items < 4 * lanes) vi = kSlab;
        }
        VP = find_variant(vi);
    }
    const Variant& V = *VP;
    if (std::strstr(V.name, "f16x3")) {  // the 16x16x32 record layout (experiment variants; built on first use)
        if (ensure_mfma16(s) != 0) return -1;
        p.mfma_frag = s->d_mfma;
        p.mfma_tau = s->d_mfma_tau;
    }
    // XCD-group item regions serve the BVH walk's L2 locality; the brute-force
    // kernels read the same records for every ray, so they take items from one
    // counter in dispatch order, which spreads neighbouring 64-pixel runs over
    // the XCDs (with <= 1 item per lane a region is one XCD's whole share: an
    // expensive band of rows would set the launch's end).  RT2_ITEM_REGIONS=0/1
    // forces the choice (A/B runs).
    static const int regions_env = [] {
        const char* e = std::getenv("RT2_ITEM_REGIONS");
        return e && *e ? std::atoi(e) : -1;
    }();
    if (regions_env == 0 || (regions_env < 0 && !is_bvh(V.kind))) p.region_ctr = nullptr;
    size_t lds = 0;
    if (V.kind == K_TILED)
        lds = (size_t)3 * sizeof(float4) * kTileTris;
    else if (V.kind == K_RESIDENT)
        lds = resident_bytes;
    else if (is_bvh(V.kind)) {
        if (V.kind == K_BVH4) p.stack_slots = std::max(s->bvh_depth, 1);  // next entry in a register
        lds = (size_t)p.stack_slots * V.block * sizeof(int);
    }
    p.bvh_recs = s->d_recs;
    p.bvh_root = s->bvh_root;
    p.recs_ok = s->recs_ok;
    s->last_kind = is_bvh(V.kind) ? K_BVH : V.kind;
    int occ = 0;
    HIPCHECK(variant_occupancy(V, &occ, lds));
    occ = std::max(occ, 1);
    unsigned long long blocks = (unsigned long long)s->num_cus * occ;
    if (V.kind == K_ASSIST || V.kind == K_MASSIST) {
        // every resident workgroup is launched: waves without items help the
        // busy waves of their workgroup.  Below 2 items per lane a quarter of
        // the waves take items (each owner has ~3 helpers; 1/4 and 1/8 slabs
        // of config B: 144 / 77 ms against 153 / 81 with half, 151 / 83 with
        // all), otherwise all of them; a chunk job has ~2 chunks per wave.
        const int nw = V.block / 64;
        const unsigned long long lanes = blocks * (unsigned long long)V.block;
        p.assist_cap = p.n_items < 2 * lanes ? std::max(1, nw / 4) : nw;
        const int g = V.kind == K_MASSIST ? 16 : 8;  // the sweep's filter group (MFMA: 16-triangle record groups)
        int chunk = (s->n_tris + 2 * nw - 1) / (2 * nw);
        chunk = std::max(g, (chunk + g - 1) / g * g);
        p.assist_chunk = chunk;
        p.assist_nchunks = s->n_tris > 0 ? (s->n_tris + chunk - 1) / chunk : 0;  // <= 2 * nw
    } else {
        const int rays_per_block = V.kind == K_SPLIT ? 64 : V.block;  // split: S waves per 64 rays
        blocks = std::min(blocks, (p.n_items + rays_per_block - 1) / rays_per_block);
    }
    blocks = std::max(blocks, 1ull);
    s->last_variant = V.id;
    HIPCHECK(V.launch(p, (int)blocks, lds, st));
    HIPCHECK(hipGetLastError());
    if (p.frame_split) {
        hipLaunchKernelGGL(frame_accumulate, dim3((unsigned)((p.n_pix + 255) / 256)), dim3(256), 0, st, p.frame_buf,
                           p.n_pix, frame_count, p.accum, p.accum8);
        HIPCHECK(hipGetLastError());
    }
    if (!s->last_launch) HIPCHECK(hipEventCreateWithFlags(&s->last_launch, hipEventDisableTiming));
    HIPCHECK(hipEventRecord(s->last_launch, st));
    s->last_launch_valid = true;
    s->samples += p.n_pix * (unsigned long long)p.R * (unsigned long long)frame_count;
    s->tests_per_seg = (unsigned long long)s->n_tris;
    return 0;
}

extern "C" int rt2_scene_stats(rt2_scene* s, rt2_stats* out, int reset) {
    if (!s || !out) {
        rt2h::set_error("rt2_scene_stats: null argument");
        return -1;
    }
    HIPCHECK(hipSetDevice(s->device));
    HIPCHECK(hipDeviceSynchronize());
    unsigned long long c[kCounters];
    HIPCHECK(hipMemcpy(c, s->d_counters, sizeof(c), hipMemcpyDeviceToHost));
    std::memcpy(s->diag, c, sizeof(c));
    out->samples = s->samples;
    out->segments = c[1];
    // brute force tests every triangle per segment; the BVH kernel counts its
    // leaf tests in c[2]
    out->tests = s->last_kind == K_BVH ? c[2] : c[1] * (unsigned long long)s->n_tris;
    out->node_visits = s->last_kind == K_BVH ? c[3] : 0;
    if (reset) {
        s->samples = 0;
        HIPCHECK(hipMemset(s->d_counters, 0, sizeof(c)));
    }
    return 0;
}

extern "C" int rt2_resolve_rgba32f(const float* d_accum, int64_t n, uint32_t frames, float* d_out, void* stream) {
    if (!d_accum || !d_out || n < 0 || frames == 0) {
        rt2h::set_error("rt2_resolve_rgba32f: bad argument");
        return -1;
    }
    if (n == 0) return 0;
    hipLaunchKernelGGL(resolve_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(d_accum), (long long)n, 0.0f, (float)frames,
                       reinterpret_cast<float4*>(d_out));
    HIPCHECK(hipGetLastError());
    return 0;
}

extern "C" int rt2_resolve_rgb8_reference(const uint32_t* acc8, int64_t n, uint32_t frames, uint8_t* out) {
    if (!acc8 || !out || n < 0 || frames == 0) {
        rt2h::set_error("rt2_resolve_rgb8_reference: bad argument");
        return -1;
    }
    const float F = (float)frames;
    for (int64_t i = 0; i < n; i++)
        for (int c = 0; c < 3; c++) {
            float v = std::min(255.0f, (float)acc8[4 * i + c] / F);
            out[3 * i + c] = (uint8_t)v;
        }
    return 0;
}

// Grows the scene's render_host buffers to `n` pixels.  On failure the
// buffers stay owned by the scene (freed by rt2_scene_destroy): no leak on any
// error path.
static int host_buffers(rt2_scene* s, size_t n) {
    if (!s->host_stream) HIPCHECK(hipStreamCreateWithFlags(&s->host_stream, hipStreamNonBlocking));
    if (n <= s->host_cap) return 0;
    HIPCHECK(hipStreamSynchronize(s->host_stream));
    (void)hipFree(s->d_host_acc);
    (void)hipFree(s->d_host_res);
    (void)hipFree(s->d_host_acc8);
    (void)hipFree(s->d_host_rgb8);
    s->d_host_acc = s->d_host_res = nullptr;
    s->d_host_acc8 = nullptr;
    s->d_host_rgb8 = nullptr;
    s->host_cap = 0;
    HIPCHECK(hipMalloc(&s->d_host_acc, n * sizeof(float4)));
    HIPCHECK(hipMalloc(&s->d_host_res, n * sizeof(float4)));
    HIPCHECK(hipMalloc(&s->d_host_acc8, n * sizeof(uint4)));
    HIPCHECK(hipMalloc(&s->d_host_rgb8, n * 3));
    s->host_cap = n;
    return 0;
}

extern "C" int rt2_render_host(rt2_scene* s, const rt2_uniforms* u, uint32_t frame_begin, uint32_t frame_count,
                               rt2_shard sh, float* out_rgba, uint8_t* out_rgb8) {
    if (!s || !u) {
        rt2h::set_error("rt2_render_host: null argument");
        return -1;
    }
    const int rows = rt2_shard_rows((int)u->height, sh);
    if (rows < 0) {
        rt2h::set_error("rt2_render_host: bad shard");
        return -1;
    }
    const size_t n = (size_t)rows * u->width;
    if (n == 0 || frame_count == 0) return 0;
    HIPCHECK(hipSetDevice(s->device));
    if (host_buffers(s, n) != 0) return -1;
    hipStream_t st = s->host_stream;
    HIPCHECK(hipMemsetAsync(s->d_host_acc, 0, n * sizeof(float4), st));
    if (out_rgb8) HIPCHECK(hipMemsetAsync(s->d_host_acc8, 0, n * sizeof(uint4), st));
    if (rt2_render(s, u, frame_begin, frame_count, sh, reinterpret_cast<float*>(s->d_host_acc),
                   out_rgb8 ? reinterpret_cast<uint32_t*>(s->d_host_acc8) : nullptr, st) != 0)
        return -1;
    if (out_rgba) {
        if (rt2_resolve_rgba32f(reinterpret_cast<const float*>(s->d_host_acc), (int64_t)n, frame_count,
                                reinterpret_cast<float*>(s->d_host_res), st) != 0)
            return -1;
        HIPCHECK(hipMemcpyAsync(out_rgba, s->d_host_res, n * sizeof(float4), hipMemcpyDeviceToHost, st));
    }
    if (out_rgb8) {
        hipLaunchKernelGGL(resolve_rgb8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           s->d_host_acc8, (long long)n, (float)frame_count, s->d_host_rgb8);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(out_rgb8, s->d_host_rgb8, n * 3, hipMemcpyDeviceToHost, st));
    }
    HIPCHECK(hipStreamSynchronize(st));  // only this render's stream, not the device
    return 0;
}

// Not in rt2.h (diagnostics): counters of the last rt2_scene_stats call
// [1] segments, [2] groups, [3] groups with survivors, [4] exact iterations,
// [5] lane survivors (STATS variants only), and the variant last launched.
// Not in rt2.h (diagnostics): all kCounters counters of the last stats call.
extern "C" int rt2_scene_diag_ex(rt2_scene* s, unsigned long long* out, int n) {
    if (!s || !out || n < 0) return -1;
    std::memcpy(out, s->diag, sizeof(unsigned long long) * (size_t)std::min(n, kCounters));
    return std::min(n, kCounters);
}

// Not in rt2.h (test hook): the cost map of the last cost-ordered launch
// (shader clocks per pixel of the slab) into `out` (n entries); returns the
// pixels it describes (0 = no valid map), < 0 on error.
extern "C" long long rt2_scene_cost_map(rt2_scene* s, uint32_t* out, unsigned long long n) {
    if (!s) return -1;
    if (!s->d_cost || s->cost_npix == 0) return 0;
    if (out && n >= s->cost_npix) {
        HIPCHECK(hipSetDevice(s->device));
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(out, s->d_cost, s->cost_npix * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    return (long long)s->cost_npix;
}

// Not in rt2.h (diagnostics): whether the scene's triangles admit sweep_plk,
// its A (max |a_i|) and how many triangles carry an always-pass record.
extern "C" int rt2_scene_plk_info(rt2_scene* s, int* ok, float* A, int* n_outside) {
    if (!s) return -1;
    if (ok) *ok = s->plk_ok;
    if (A) *A = s->plk_A;
    if (n_outside) *n_outside = s->plk_outside;
    return 0;
}

extern "C" int rt2_scene_diag(rt2_scene* s, unsigned long long* out8, int* last_variant) {
    if (!s || !out8) return -1;
    std::memcpy(out8, s->diag, 8 * sizeof(unsigned long long));
    if (last_variant) *last_variant = s->last_variant;
    return 0;
}

// Not in rt2.h (test hook): exhaustive reciprocal check over [lo, hi] bit patterns.
extern "C" int rt2_device_rcp_check(uint32_t lo, uint32_t hi, int variant, unsigned long long* mismatches,
                                    uint32_t* first_bad) {
    unsigned long long* d = nullptr;
    HIPCHECK(hipMalloc(&d, 16));
    HIPCHECK(hipMemset(d, 0, 8));
    uint32_t init = 0xffffffffu;
    HIPCHECK(hipMemcpy((char*)d + 8, &init, 4, hipMemcpyHostToDevice));
    const unsigned long long count = (unsigned long long)hi - lo + 1;
    hipLaunchKernelGGL(rcp_check_kernel, dim3(4096), dim3(256), 0, 0, lo, count, variant, d, (uint32_t*)((char*)d + 8));
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpy(mismatches, d, 8, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(first_bad, (char*)d + 8, 4, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

// Not in rt2.h (test hook): div_mk (mode 0) or div64 (mode 1) against IEEE
// division on `count` random (n, d) pairs of the ranges the kernels use them on.
extern "C" int rt2_device_div_check(uint32_t seed, unsigned long long count, int mode,
                                    unsigned long long* mismatches, uint32_t* first_bad) {
    unsigned long long* d = nullptr;
    HIPCHECK(hipMalloc(&d, 16));
    HIPCHECK(hipMemset(d, 0, 8));
    uint32_t init = 0xffffffffu;
    HIPCHECK(hipMemcpy((char*)d + 8, &init, 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(div_check_kernel, dim3(8192), dim3(256), 0, 0, seed, count, mode, d,
                       (uint32_t*)((char*)d + 8));
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpy(mismatches, d, 8, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(first_bad, (char*)d + 8, 4, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

// Not in rt2.h (test hook): device numerics self-test, host in/out arrays.
extern "C" int rt2_device_selftest(const float* in, int32_t n, float* out10) {
    float *din = nullptr, *dout = nullptr;
    HIPCHECK(hipMalloc(&din, (size_t)n * 4));
    HIPCHECK(hipMalloc(&dout, (size_t)n * 40));
    HIPCHECK(hipMemcpy(din, in, (size_t)n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, din, n, dout);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpy(out10, dout, (size_t)n * 40, hipMemcpyDeviceToHost));
    (void)hipFree(din);
    (void)hipFree(dout);
    return 0;
}

// Not in rt2.h (test hook): copies one of the scene's derived device arrays to
// host memory: 0 = pre-transformed triangles (3 float4 each), 1 = render_mfma
// records (16x16x32 layout), 2 = their per-triangle tau, 3 = sweep_k16 records,
// 4 = their tau, 5 = the k5 form's per-triangle m.z residual bounds, 6 = the
// kthr records (threshold in the K-slots).  Returns the array's size in bytes (nothing copied when
// `host` is null or `bytes` is too small), < 0 on error.
extern "C" long long rt2_scene_export(rt2_scene* s, int what, void* host, unsigned long long bytes) {
    if (!s) return -1;
    const size_t n = (size_t)std::max(s->n_tris, 1), n16 = (size_t)(s->n_tris + 15) / 16 * 16,
                 n32 = (size_t)(s->n_tris + 31) / 32 * 32;
    const void* src = nullptr;
    size_t sz = 0;
    if ((what == 1 || what == 2) && ensure_mfma16(s) != 0) return -1;
    switch (what) {
    case 0: src = s->d_tri, sz = n * 3 * sizeof(float4); break;
    case 1: src = s->d_mfma, sz = n16 * kMfmaQ * 32 * sizeof(_Float16); break;
    case 2: src = s->d_mfma_tau, sz = n16 * sizeof(float); break;
    case 3: src = s->d_mfma_k16, sz = n32 * kK16Ops * 16 * sizeof(_Float16); break;
    case 4: src = s->d_mfma_k16_tau, sz = n32 * sizeof(float); break;
    case 5: src = s->d_mfma_k16_bnd, sz = n32 * sizeof(float2); break;
    case 6: src = s->d_mfma_kt, sz = n32 * kKtOps * 16 * sizeof(_Float16); break;
    default: return -1;
    }
    if (!src || s->n_tris == 0) return 0;
    if (host && bytes >= sz) {
        HIPCHECK(hipSetDevice(s->device));
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(host, src, sz, hipMemcpyDeviceToHost));
    }
    return (long long)sz;
}

// Not in rt2.h (test hook): the matrix filter's terms on the hardware
// (mfma_probe_kernel) for n_rays rays (a multiple of 64; 8 floats each: o.xyz,
// best, d.xyz, 0) against every triangle of the scene.  layout 0 = the
// 16x16x32 form of render_mfma (variants 150/152), 1 = the k16 form
// (sweep_k16), 2 = its 5-product form (MfmaSpec::k5: U, -V, X from the first
// K-half), 3 = the 5-product form with the threshold in the accumulator
// (MfmaSpec::cthr: U, -V, X, Y shifted by TT = -Tl'', TT in the -tn slot),
// 4 = layout 3 with the fragments built in registers by frag_pair (the
// operand path of 282 / 293 / 298), 5 = the threshold in the K-slots
// (MfmaSpec::kthr, frag_pair fragments: U, -V, X, Y, slot 3 zero), 6 = layout
// 5 with each ray's own W (MfmaSpec::kt_lane_w).
// Host outputs, sized by the caller: terms [n_rays][n_pad][5]
// (n_pad = triangles padded to 16 / 32), frags [n_rays][80] f16 bits (the LDS
// row of layouts 0..3: main slots 0..31 and Y slots 16..31; layouts 4, 5 also
// the register fragments the MFMA read: main K-half at 48..63, Y at 64..79),
// rinfo [n_rays][8], accept [n_rays][n_tris].
extern "C" int rt2_mfma_probe(rt2_scene* s, int layout, const float* rays, int32_t n_rays, float* terms,
                              uint16_t* frags, float* rinfo, uint8_t* accept) {
    if (!s || !rays || n_rays <= 0 || n_rays % 64 != 0 || !terms || !frags || !rinfo || !accept ||
        layout < 0 || layout > 6 || s->n_tris < 1 || !s->mfma_ok) {
        rt2h::set_error("rt2_mfma_probe: bad argument (n_rays a positive multiple of 64, a scene in the filter's "
                        "range)");
        return -1;
    }
    HIPCHECK(hipSetDevice(s->device));
    if (layout == 0 && ensure_mfma16(s) != 0) return -1;
    const int n_pad = layout >= 1 ? (s->n_tris + 31) / 32 * 32 : (s->n_tris + 15) / 16 * 16;
    const size_t nr = (size_t)n_rays;
    const size_t b_rays = nr * 8 * sizeof(float), b_terms = nr * n_pad * 5 * sizeof(float),
                 b_frags = nr * 80 * sizeof(uint16_t), b_info = nr * 8 * sizeof(float), b_acc = nr * s->n_tris;
    char* d = nullptr;
    HIPCHECK(hipMalloc(&d, b_rays + b_terms + b_frags + b_info + b_acc + 64));
    char* p0 = d;
    float4* d_rays = (float4*)p0;
    float* d_terms = (float*)(p0 += b_rays);
    _Float16* d_frags = (_Float16*)(p0 += b_terms);
    float* d_info = (float*)(p0 += b_frags);
    uint8_t* d_acc = (uint8_t*)(p0 += b_info);
    int rc = 0;
    auto run = [&]() -> int {
        HIPCHECK(hipMemcpy(d_rays, rays, b_rays, hipMemcpyHostToDevice));
        HIPCHECK(hipMemset(d_terms, 0, b_terms));
        RenderParams p;
        std::memset(&p, 0, sizeof(p));
        p.tri = s->d_tri;
        p.n_tris = s->n_tris;
        p.mfma_frag = s->d_mfma;
        p.mfma_tau = s->d_mfma_tau;
        p.mfma_A = s->mfma_A;
        p.mfma_k16_frag = s->d_mfma_k16;
        p.mfma_k16_tau = s->d_mfma_k16_tau;
        p.mfma_k16_bnd = s->d_mfma_k16_bnd;
        p.mfma_kt_frag = s->d_mfma_kt;
        constexpr MfmaSpec k16 = k16_spec(3), f16x32 = kMfmaT8Y4;
        constexpr MfmaSpec k5 = [] {
            MfmaSpec x = k16_spec(3);
            x.k5 = true;
            return x;
        }();
        constexpr MfmaSpec k5c = [] {
            MfmaSpec x = k16_spec(3);
            x.k5 = true;
            x.no_tn = true;
            x.cthr = true;
            return x;
        }();
        // the shipping operand path: fragments by frag_pair (v_permlane32_swap), cthr (282 / 293 / 298) or
        // kthr (the threshold in the K-slots)
        constexpr MfmaSpec k5cp = [] {
            MfmaSpec x = k5_res_spec(4);
            x.perm_frag = true;
            return x;
        }();
        constexpr MfmaSpec ktp = [] {
            MfmaSpec x = kt_res_spec(1);
            x.perm_frag = true;
            return x;
        }();
        constexpr MfmaSpec ktpl = [] {
            MfmaSpec x = kt_res_spec(1);
            x.perm_frag = true;
            x.kt_lane_w = true;
            return x;
        }();
        if (layout == 4)
            hipLaunchKernelGGL(mfma_probe_kernel<k5cp>, dim3(n_rays / 64), dim3(64), 0, 0, p, d_rays, n_pad, d_terms,
                               d_frags, d_info, d_acc);
        else if (layout == 5)
            hipLaunchKernelGGL(mfma_probe_kernel<ktp>, dim3(n_rays / 64), dim3(64), 0, 0, p, d_rays, n_pad, d_terms,
                               d_frags, d_info, d_acc);
        else if (layout == 6)
            hipLaunchKernelGGL(mfma_probe_kernel<ktpl>, dim3(n_rays / 64), dim3(64), 0, 0, p, d_rays, n_pad, d_terms,
                               d_frags, d_info, d_acc);
        else if (layout == 3)
            hipLaunchKernelGGL(mfma_probe_kernel<k5c>, dim3(n_rays / 64), dim3(64), 0, 0, p, d_rays, n_pad, d_terms,
                               d_frags, d_info, d_acc);
        else if (layout == 1)
            hipLaunchKernelGGL(mfma_probe_kernel<k16>, dim3(n_rays / 64), dim3(64), 0, 0, p, d_rays, n_pad, d_terms,
                               d_frags, d_info, d_acc);
        else if (layout == 2)
            hipLaunchKernelGGL(mfma_probe_kernel<k5>, dim3(n_rays / 64), dim3(64), 0, 0, p, d_rays, n_pad, d_terms,
                               d_frags, d_info, d_acc);
        else
            hipLaunchKernelGGL(mfma_probe_kernel<f16x32>, dim3(n_rays / 64), dim3(64), 0, 0, p, d_rays, n_pad,
                               d_terms, d_frags, d_info, d_acc);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(terms, d_terms, b_terms, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(frags, d_frags, b_frags, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(rinfo, d_info, b_info, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(accept, d_acc, b_acc, hipMemcpyDeviceToHost));
        return 0;
    };
    rc = run();
    (void)hipFree(d);
    return rc;
}
