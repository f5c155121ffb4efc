// Multi-GPU half of the C-ABI (include/rt2.h, "Multi-GPU"): row-tile shards of
// one image rendered by one process per GPU, brought to a root rank by ONE
// RCCL gather over xGMI, un-interleaved on the root.
//
// The reference renders on one GPU and reads the framebuffer back with
// glReadPixels (RayTracing/src/rayTracing.cpp:217) inside screenshot()
// (:124-283); rt2_render_host_gather is that readback for N ranks: every rank
// renders its slab (rt2_render), resolves it on its device, and the resolved
// slabs travel to the root in one ncclGather (rccl.h ncclGather), which then
// holds the whole image — bit-identical to a one-GPU render, since every
// pixel's arithmetic is independent of the shard that renders it.
//
// Host code only, apart from the un-interleave and 8-bit resolve kernels.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "../../../include/rt2.h"

namespace rt2h {
void set_error(const std::string& msg);
}

static_assert(sizeof(ncclUniqueId) == RT2_COMM_ID_BYTES, "RT2_COMM_ID_BYTES must equal sizeof(ncclUniqueId)");

#define HIPCHECK(expr)                                                                         \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            rt2h::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                \
            return -1;                                                                         \
        }                                                                                      \
    } while (0)
#define NCCLCHECK(expr)                                                                        \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess) {                                                               \
            rt2h::set_error(std::string(#expr) + ": " + ncclGetErrorString(r_));               \
            return -1;                                                                         \
        }                                                                                      \
    } while (0)

namespace {

// One 16-byte element per pixel (float4 colour or uint4 8-bit sums).
// Image pixel (y, x) comes from slab row lr of rank r in the gathered buffer
// [nranks][max_rows][W]: r = (y / tile) % n, lr = (y / tile / n) * tile + y % tile
// (the inverse of rt2_shard_row).
__global__ void unshard_kernel(const uint4* __restrict__ gathered, int max_rows, int W, int H, int tile, int n,
                               uint4* __restrict__ image) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)W * H) return;
    const int y = (int)(i / W), x = (int)(i - (long long)y * W);
    const int t = y / tile;
    const int r = t % n;
    const int lr = (t / n) * tile + y % tile;
    image[i] = gathered[((long long)r * max_rows + lr) * W + x];
}

// rayTracing.cpp:248-250 on the device (same operations as the host
// rt2_resolve_rgb8_reference).
__global__ void rgb8_kernel(const uint4* acc8, long long n, float frames, uint8_t* out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 q = acc8[i];
    out[3 * i + 0] = (uint8_t)fminf(255.0f, (float)q.x / frames);
    out[3 * i + 1] = (uint8_t)fminf(255.0f, (float)q.y / frames);
    out[3 * i + 2] = (uint8_t)fminf(255.0f, (float)q.z / frames);
}

// A device buffer that only grows; freed by the owning communicator.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        (void)hipFree(p);
        p = nullptr;
        cap = 0;
        HIPCHECK(hipMalloc(&p, std::max<size_t>(bytes, 16)));
        cap = bytes;
        return 0;
    }
    void release() {
        (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

int max_slab_rows(int height, rt2_shard sh) {
    int m = 0;
    for (int r = 0; r < sh.nranks; r++) m = std::max(m, rt2_shard_rows(height, rt2_shard{sh.tile_rows, r, sh.nranks}));
    return m;
}

}  // namespace

struct rt2_comm {
    ncclComm_t comm = nullptr;
    bool owned = false;
    bool aborted = false;          // a rank-local failure aborted the communicator (owned ones only)
    int nranks = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;  // rt2_render_host_gather's stream
    DevBuf send, gathered;         // rt2_gather_slabs: padded send slab, root's [nranks][max_rows][W]
    DevBuf acc, res, acc8;         // rt2_render_host_gather: this rank's slab (max_rows rows)
    DevBuf hgathered;              // rt2_render_host_gather: root's [nranks][max_rows][W] (not shared with
                                   // rt2_gather_slabs, whose use may still be in flight on another stream)
    DevBuf image, image8, rgb8;    // rt2_render_host_gather: root's whole image
    DevBuf status;                 // rt2_render_host_gather: the ranks' agreement words (int32 x 2)
};

extern "C" int rt2_comm_unique_id(uint8_t* id) {
    if (!id) {
        rt2h::set_error("rt2_comm_unique_id: null argument");
        return -1;
    }
    ncclUniqueId u;
    NCCLCHECK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return 0;
}

static int comm_setup(rt2_comm* c) {
    int n = 0, r = 0;
    NCCLCHECK(ncclCommCount(c->comm, &n));
    NCCLCHECK(ncclCommUserRank(c->comm, &r));
    c->nranks = n;
    c->rank = r;
    HIPCHECK(hipSetDevice(c->device));
    HIPCHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    return c->status.ensure(2 * sizeof(int32_t));  // allocated up front: the agreement step cannot fail on memory
}

// Every rank calls the same collectives in the same order, whatever happened
// locally: a rank that returned early would leave its peers blocked in the
// next collective.  agree_max is rt2_render_host_gather's agreement step (one
// 2-int ncclAllReduce(max) on the communicator's stream, read back on the
// host): v[0] = "this rank failed", v[1] = "this rank wants the 8-bit sums".
static int agree_max(rt2_comm* c, int32_t v[2]) {
    HIPCHECK(hipMemcpyAsync(c->status.p, v, 2 * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    NCCLCHECK(ncclAllReduce(c->status.p, c->status.p, 2, ncclInt32, ncclMax, c->comm, c->stream));
    HIPCHECK(hipMemcpyAsync(v, c->status.p, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    return 0;
}

// A rank-local failure inside rt2_gather_slabs (asynchronous, so there is no
// agreement step): an owned communicator is aborted so that the peers' gather
// fails instead of blocking forever; it is unusable afterwards (destroy it).  A
// wrapped communicator belongs to the caller and is left to the caller's abort.
static int fail_collective(rt2_comm* c, const std::string& msg) {
    if (c->owned && c->comm && !c->aborted) {
        (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
        c->aborted = true;
        rt2h::set_error(msg + " (communicator aborted so that the peer ranks fail instead of blocking)");
    } else {
        rt2h::set_error(msg);
    }
    return -1;
}

extern "C" int rt2_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, rt2_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks || device < 0) {
        rt2h::set_error("rt2_comm_init: bad argument");
        return -1;
    }
    HIPCHECK(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    rt2_comm* c = new rt2_comm();
    c->device = device;
    c->owned = true;
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        rt2h::set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        c->comm = nullptr;
        rt2_comm_destroy(c);
        return -1;
    }
    if (comm_setup(c) != 0) {
        rt2_comm_destroy(c);
        return -1;
    }
    *out = c;
    return 0;
}

extern "C" int rt2_comm_wrap(void* nccl_comm, int32_t device, rt2_comm** out) {
    if (!nccl_comm || !out || device < 0) {
        rt2h::set_error("rt2_comm_wrap: bad argument");
        return -1;
    }
    rt2_comm* c = new rt2_comm();
    c->comm = (ncclComm_t)nccl_comm;
    c->device = device;
    c->owned = false;
    if (comm_setup(c) != 0) {
        rt2_comm_destroy(c);
        return -1;
    }
    *out = c;
    return 0;
}

extern "C" void rt2_comm_destroy(rt2_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    for (DevBuf* b : {&c->send, &c->gathered, &c->acc, &c->res, &c->acc8, &c->hgathered, &c->image, &c->image8,
                      &c->rgb8, &c->status})
        b->release();
    if (c->owned && c->comm) (void)ncclCommDestroy(c->comm);  // null after an abort
    delete c;
}

extern "C" int rt2_comm_check(rt2_comm* c) {
    if (!c) {
        rt2h::set_error("rt2_comm_check: null communicator");
        return -1;
    }
    if (c->aborted) {
        rt2h::set_error("rt2_comm_check: the communicator was aborted after a rank-local failure");
        return -1;
    }
    ncclResult_t async = ncclSuccess;
    NCCLCHECK(ncclCommGetAsyncError(c->comm, &async));
    if (async != ncclSuccess) {
        rt2h::set_error(std::string("RCCL asynchronous error: ") + ncclGetErrorString(async));
        return -1;
    }
    return 0;
}

extern "C" int rt2_comm_size(rt2_comm* c, int32_t* nranks, int32_t* rank) {
    if (!c) {
        rt2h::set_error("rt2_comm_size: null communicator");
        return -1;
    }
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return 0;
}

extern "C" int rt2_unshard_slabs(const void* d_gathered, int32_t max_rows, int32_t width, int32_t height,
                                 rt2_shard layout, void* d_image, void* stream) {
    if (!d_gathered || !d_image || width < 1 || height < 0 || layout.tile_rows < 1 || layout.nranks < 1 ||
        max_rows < max_slab_rows(height, layout)) {
        rt2h::set_error("rt2_unshard_slabs: bad argument");
        return -1;
    }
    const long long n = (long long)width * height;
    if (n == 0) return 0;
    hipLaunchKernelGGL(unshard_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)d_gathered, max_rows, width, height, layout.tile_rows, layout.nranks,
                       (uint4*)d_image);
    HIPCHECK(hipGetLastError());
    return 0;
}

extern "C" int rt2_gather_slabs(rt2_comm* c, const void* d_slab, int32_t width, int32_t height, rt2_shard sh,
                                int32_t root, void* d_image, void* stream) {
    // argument errors every rank sees alike (the same width/height/root/layout
    // are passed everywhere): nothing is issued, as on every peer
    if (!c || width < 1 || height < 0 || root < 0 || root >= c->nranks) {
        rt2h::set_error("rt2_gather_slabs: bad argument");
        return -1;
    }
    if (rt2_comm_check(c) != 0) return -1;  // aborted, or a collective failed earlier on this communicator
    if (sh.nranks != c->nranks || sh.rank != c->rank || rt2_shard_rows(height, sh) < 0)
        return fail_collective(c, "rt2_gather_slabs: shard " + std::to_string(sh.rank) + "/" +
                                      std::to_string(sh.nranks) + " does not match the communicator's rank " +
                                      std::to_string(c->rank) + "/" + std::to_string(c->nranks));
    if (!d_slab) return fail_collective(c, "rt2_gather_slabs: null slab");
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    const int rows = rt2_shard_rows(height, sh), mr = max_slab_rows(height, sh);
    const size_t slab_bytes = (size_t)mr * width * 16;
    const void* send = d_slab;
    if (rows < mr) {  // equal counts per rank: pad this slab to max_rows rows
        if (c->send.ensure(slab_bytes) != 0) return fail_collective(c, "rt2_gather_slabs: out of device memory");
        HIPCHECK(hipMemsetAsync(c->send.p, 0, slab_bytes, st));
        HIPCHECK(hipMemcpyAsync(c->send.p, d_slab, (size_t)rows * width * 16, hipMemcpyDeviceToDevice, st));
        send = c->send.p;
    }
    // a root without d_image still takes part (into the scratch buffer), then fails
    const bool is_root = c->rank == root, root_ok = !is_root || d_image;
    void* recv = nullptr;
    if (is_root) {
        if (c->nranks == 1 && d_image) {
            recv = d_image;  // the slab is the image
        } else {
            if (c->gathered.ensure(slab_bytes * c->nranks) != 0)
                return fail_collective(c, "rt2_gather_slabs: out of device memory");
            recv = c->gathered.p;
        }
    }
    NCCLCHECK(ncclGather(send, recv, slab_bytes, ncclUint8, root, c->comm, st));
    if (!root_ok) {
        rt2h::set_error("rt2_gather_slabs: the root needs d_image");
        return -1;
    }
    if (is_root && c->nranks > 1) return rt2_unshard_slabs(c->gathered.p, mr, width, height, sh, d_image, st);
    return 0;
}

extern "C" int rt2_render_host_gather(rt2_scene* scene, const rt2_uniforms* u, uint32_t frame_begin,
                                      uint32_t frame_count, rt2_shard sh, rt2_comm* c, int32_t root, float* out_rgba,
                                      uint8_t* out_rgb8) {
    if (!c || !u || root < 0 || root >= c->nranks) {  // seen alike on every rank: nothing issued
        rt2h::set_error("rt2_render_host_gather: bad argument");
        return -1;
    }
    if (rt2_comm_check(c) != 0) return -1;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const int H = (int)u->height, W = (int)u->width;
    const bool is_root = c->rank == root;
    // Rank-local failures do not return before the agreement steps below: every
    // rank issues the same collectives, then all fail together.
    std::string err;
    if (!scene || frame_count == 0 || W < 1 || H < 0)
        err = "rt2_render_host_gather: bad argument";
    else if (sh.nranks != c->nranks || sh.rank != c->rank || rt2_shard_rows(H, sh) < 0)
        err = "rt2_render_host_gather: shard does not match the communicator";
    // agreement 1: the 8-bit sums are accumulated and gathered when any rank
    // asks for them (the root's out_rgb8 receives them), so the collective
    // sequence never depends on one rank's pointers
    int32_t v[2] = {err.empty() ? 0 : 1, out_rgb8 ? 1 : 0};
    if (agree_max(c, v) != 0) return -1;
    if (v[0]) {
        rt2h::set_error(err.empty() ? "rt2_render_host_gather: a peer rank failed" : err);
        return -1;
    }
    const bool rgb8 = v[1] != 0;
    const int mr = max_slab_rows(H, sh);
    const size_t slab = (size_t)mr * W * 16, whole = (size_t)W * H;
    const int rows = rt2_shard_rows(H, sh);
    auto local = [&]() -> int {
        if (c->acc.ensure(slab) || c->res.ensure(slab) || (rgb8 && c->acc8.ensure(slab))) return -1;
        if (is_root && (c->image.ensure(whole * 16) || (rgb8 && (c->image8.ensure(whole * 16) ||
                                                                  c->rgb8.ensure(whole * 3)))))
            return -1;
        if (is_root && c->nranks > 1 && c->hgathered.ensure(slab * c->nranks)) return -1;
        // slab buffers of max_rows rows, zeroed: the rows past this rank's slab
        // are the gather's padding
        HIPCHECK(hipMemsetAsync(c->acc.p, 0, slab, st));
        HIPCHECK(hipMemsetAsync(c->res.p, 0, slab, st));
        if (rgb8) HIPCHECK(hipMemsetAsync(c->acc8.p, 0, slab, st));
        if (rt2_render(scene, u, frame_begin, frame_count, sh, (float*)c->acc.p,
                       rgb8 ? (uint32_t*)c->acc8.p : nullptr, st) != 0)
            return -1;
        if (rt2_resolve_rgba32f((const float*)c->acc.p, (int64_t)rows * W, frame_count, (float*)c->res.p, st) != 0)
            return -1;
        return 0;
    };
    // agreement 2: every rank rendered (errors on the stream surface at the
    // agreement's synchronisation)
    const int lrc = local();
    const std::string lerr = lrc != 0 ? std::string(rt2_last_error()) : std::string();
    v[0] = lrc != 0 ? 1 : 0;
    v[1] = 0;
    if (agree_max(c, v) != 0) return -1;
    if (v[0]) {
        rt2h::set_error(lrc != 0 ? lerr : std::string("rt2_render_host_gather: a peer rank failed"));
        return -1;
    }
    void* recv = is_root ? (c->nranks == 1 ? c->image.p : c->hgathered.p) : nullptr;
    NCCLCHECK(ncclGather(c->res.p, recv, slab, ncclUint8, root, c->comm, st));
    if (is_root && c->nranks > 1 && rt2_unshard_slabs(c->hgathered.p, mr, W, H, sh, c->image.p, st) != 0) return -1;
    if (rgb8) {
        void* recv8 = is_root ? (c->nranks == 1 ? c->image8.p : c->hgathered.p) : nullptr;
        NCCLCHECK(ncclGather(c->acc8.p, recv8, slab, ncclUint8, root, c->comm, st));
        if (is_root && c->nranks > 1 && rt2_unshard_slabs(c->hgathered.p, mr, W, H, sh, c->image8.p, st) != 0)
            return -1;
        if (is_root && out_rgb8) {
            hipLaunchKernelGGL(rgb8_kernel, dim3((unsigned)((whole + 255) / 256)), dim3(256), 0, st,
                               (const uint4*)c->image8.p, (long long)whole, (float)frame_count, (uint8_t*)c->rgb8.p);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipMemcpyAsync(out_rgb8, c->rgb8.p, whole * 3, hipMemcpyDeviceToHost, st));
        }
    }
    if (is_root && out_rgba) HIPCHECK(hipMemcpyAsync(out_rgba, c->image.p, whole * 16, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    return rt2_comm_check(c);
}
