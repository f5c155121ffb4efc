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
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "../../../include/rt2.h"
#include "rt2_comm_protocol.h"

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
    DevBuf status;                 // the agreement words (int32 x 2) on the device
    int32_t* hstatus = nullptr;    // ... and in pinned host memory (copies that never block the host)
    hipEvent_t pre_gather = nullptr;       // rt2_gather_slabs: recorded on the caller's stream right before the
    hipStream_t pre_gather_st = nullptr;   // gather, so rt2_comm_wait can tell this rank's own queued work (the
    bool pre_gather_valid = false;         // render) from the collective
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
    HIPCHECK(hipHostMalloc((void**)&c->hstatus, 2 * sizeof(int32_t), hipHostMallocDefault));
    return c->status.ensure(2 * sizeof(int32_t));  // allocated up front: the agreement step cannot fail on memory
}

namespace {

// Deadline of every host wait on a collective (RT2_COMM_TIMEOUT_S, default
// 600 s: the agreement after the render also waits for the slowest rank's
// render).
double comm_timeout_s() {
    const char* e = std::getenv("RT2_COMM_TIMEOUT_S");
    const double v = e && *e ? std::atof(e) : 0.0;
    return v > 0.0 ? v : 600.0;
}

// RCCL transport of the gather protocol (rt2_comm_protocol.h).  Fault
// injection for the failure tests: RT2_FAULT_AT=<site>[@rank] makes this rank
// (every rank without @rank) fail at that site — gather.prepare,
// gather.issue, check, render (the protocol's sites) or agree.copy (this
// transport's: the rank cannot take part in the agreement at all).
struct RcclTransport {
    rt2_comm* c;
    double slack_s = 0.0;  // added to the deadline: 2x this rank's own render time (the peers render alike)
    bool usable() const { return c->comm && !c->aborted; }
    bool fault(const char* site) const {
        const char* e = std::getenv("RT2_FAULT_AT");
        if (!e || !*e) return false;
        const std::string f(e);
        const size_t at = f.find('@');
        if (f.substr(0, at) != site) return false;
        return at == std::string::npos || std::atoi(f.c_str() + at + 1) == c->rank;
    }
    // an owned communicator is aborted (ncclCommAbort); a wrapped one belongs to
    // the caller, who has to abort it: this handle only refuses further use
    void abort(const std::string& why) {
        if (c->owned && c->comm && !c->aborted) {
            (void)ncclCommAbort(c->comm);
            c->comm = nullptr;
        }
        c->aborted = true;
        rt2h::set_error("rt2 comm: " + why + (c->owned ? " (communicator aborted)" : " (abort the wrapped communicator)"));
    }
    // the host waits for stream `st` with a deadline: a collective whose peer
    // never joins it is aborted there instead of blocking forever
    int wait(hipStream_t st) {
        const auto t0 = std::chrono::steady_clock::now();
        const double limit = comm_timeout_s() + slack_s;
        for (;;) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) return 0;
            if (q != hipErrorNotReady) {
                abort(std::string("stream error while waiting for a collective: ") + hipGetErrorString(q));
                return -1;
            }
            ncclResult_t a = ncclSuccess;
            if (c->comm && ncclCommGetAsyncError(c->comm, &a) == ncclSuccess && a != ncclSuccess &&
                a != ncclInProgress) {
                abort(std::string("RCCL asynchronous error: ") + ncclGetErrorString(a));
                return -1;
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
                abort("a peer rank did not join the collective within RT2_COMM_TIMEOUT_S");
                return -1;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    // this rank's own work on stream `st` (no collective in it, so no peer can
    // hold it up): waited for without a deadline, and its duration becomes
    // slack on the deadlines that follow — the next agreement also waits for
    // the slowest peer's render of an equal slab
    // The local wait is still bounded (a kernel that never finishes must not
    // hang this host forever while the peers time out): 20x RT2_COMM_TIMEOUT_S,
    // then abort; a stream error aborts with HIP's message.
    template <class Query>
    int wait_local_q(Query query) {
        const auto t0 = std::chrono::steady_clock::now();
        const double limit = 20.0 * comm_timeout_s();
        for (;;) {
            const hipError_t q = query();
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) {
                abort(std::string("stream error in this rank's own work before a collective: ") + hipGetErrorString(q));
                return -1;
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
                abort("this rank's own work before a collective ran longer than 20 x RT2_COMM_TIMEOUT_S");
                return -1;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        slack_s = 2.0 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return 0;
    }
    int wait_local(hipStream_t st) {
        return wait_local_q([&] { return hipStreamQuery(st); });
    }
    int wait_local_event(hipEvent_t ev) {
        return wait_local_q([&] { return hipEventQuery(ev); });
    }
    // the agreement step: allreduce(max) of two ints on the communicator's own
    // stream, read back into pinned memory and waited for under the deadline;
    // any failure of this rank's part aborts
    int agree(int32_t v[2]) {
        if (!usable()) return -1;
        c->hstatus[0] = v[0];
        c->hstatus[1] = v[1];
        if (fault("agree.copy") ||
            hipMemcpyAsync(c->status.p, c->hstatus, 2 * sizeof(int32_t), hipMemcpyHostToDevice, c->stream) !=
                hipSuccess) {
            abort("the agreement's copy failed");
            return -1;
        }
        if (ncclAllReduce(c->status.p, c->status.p, 2, ncclInt32, ncclMax, c->comm, c->stream) != ncclSuccess) {
            abort("the agreement's allreduce could not be issued");
            return -1;
        }
        if (hipMemcpyAsync(c->hstatus, c->status.p, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess) {
            abort("the agreement's copy failed");
            return -1;
        }
        if (wait(c->stream) != 0) return -1;
        v[0] = c->hstatus[0];
        v[1] = c->hstatus[1];
        return 0;
    }
};

}  // namespace

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
    if (c->hstatus) (void)hipHostFree(c->hstatus);
    if (c->pre_gather) (void)hipEventDestroy(c->pre_gather);
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
    hipStream_t st = (hipStream_t)stream;
    const bool is_root = c->rank == root;
    int mr = 0;
    size_t slab_bytes = 0;
    const void* send = d_slab;
    void* recv = nullptr;
    // this rank's checks, padding and receive buffer: a failure here is agreed
    // on before the gather, so every rank returns < 0 and none issues it
    auto prepare = [&](std::string& err) -> int {
        if (hipSetDevice(c->device) != hipSuccess) return err = "hipSetDevice failed", -1;
        if (sh.nranks != c->nranks || sh.rank != c->rank || rt2_shard_rows(height, sh) < 0) {
            err = "shard " + std::to_string(sh.rank) + "/" + std::to_string(sh.nranks) +
                  " does not match the communicator's rank " + std::to_string(c->rank) + "/" +
                  std::to_string(c->nranks);
            return -1;
        }
        if (!d_slab) return err = "null slab", -1;
        if (is_root && !d_image) return err = "the root needs d_image", -1;
        const int rows = rt2_shard_rows(height, sh);
        mr = max_slab_rows(height, sh);
        slab_bytes = (size_t)mr * width * 16;
        if (rows < mr) {  // equal counts per rank: pad this slab to max_rows rows
            if (c->send.ensure(slab_bytes) != 0) return err = "out of device memory", -1;
            if (hipMemsetAsync(c->send.p, 0, slab_bytes, st) != hipSuccess ||
                hipMemcpyAsync(c->send.p, d_slab, (size_t)rows * width * 16, hipMemcpyDeviceToDevice, st) !=
                    hipSuccess)
                return err = "the padding copy failed", -1;
            send = c->send.p;
        }
        if (is_root) {
            if (c->nranks == 1) {
                recv = d_image;  // the slab is the image
            } else {
                if (c->gathered.ensure(slab_bytes * c->nranks) != 0) return err = "out of device memory", -1;
                recv = c->gathered.p;
            }
        }
        return 0;
    };
    auto gather = [&]() -> int {
        // everything queued on `st` before this point is this rank's own work
        // (the render, the padding copy): rt2_comm_wait waits for it without
        // the collective's deadline
        if (!c->pre_gather && hipEventCreateWithFlags(&c->pre_gather, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventRecord(c->pre_gather, st) != hipSuccess) return -1;
        c->pre_gather_st = st;
        c->pre_gather_valid = true;
        return ncclGather(send, recv, slab_bytes, ncclUint8, root, c->comm, st) == ncclSuccess ? 0 : -1;
    };
    auto finish = [&](std::string& err) -> int {
        if (is_root && c->nranks > 1 && rt2_unshard_slabs(c->gathered.p, mr, width, height, sh, d_image, st) != 0)
            return err = rt2_last_error(), -1;
        return 0;
    };
    RcclTransport t{c};
    // The rank's own work already queued on `stream` (its render) is waited
    // for first, without the collective's deadline (bounded at 20x it), and
    // twice its duration becomes slack on the deadlines that follow: the
    // agreement's allreduce cannot start on a device still busy with the
    // render, so a render longer than RT2_COMM_TIMEOUT_S would otherwise
    // abort a healthy job at the agreement
    if (hipSetDevice(c->device) != hipSuccess) {
        rt2h::set_error("rt2_gather_slabs: hipSetDevice failed");
        return -1;
    }
    if (!c->aborted && c->comm) {
        if ((!c->pre_gather && hipEventCreateWithFlags(&c->pre_gather, hipEventDisableTiming) != hipSuccess) ||
            hipEventRecord(c->pre_gather, st) != hipSuccess) {
            rt2h::set_error("rt2_gather_slabs: could not record the render's event");
            return -1;
        }
        if (t.wait_local_event(c->pre_gather) != 0) return -1;  // aborted, error set
    }
    std::string err;
    if (rt2p::gather_slabs(t, prepare, gather, finish, err) != 0) {
        rt2h::set_error("rt2_gather_slabs: " + err);
        return -1;
    }
    return 0;
}

extern "C" int rt2_comm_wait(rt2_comm* c, void* stream) {
    if (!c) {
        rt2h::set_error("rt2_comm_wait: null communicator");
        return -1;
    }
    if (c->aborted) {
        rt2h::set_error("rt2_comm_wait: the communicator was aborted after a rank-local failure");
        return -1;
    }
    HIPCHECK(hipSetDevice(c->device));
    RcclTransport t{c};
    // the rank's own work queued before the last gather on this stream (its
    // render: peers render alike) is waited for first, bounded but outside the
    // deadline, and its duration becomes slack (a render longer than
    // RT2_COMM_TIMEOUT_S must not abort a healthy job); then the deadline
    // applies to the gather itself
    if (c->pre_gather_valid && c->pre_gather_st == (hipStream_t)stream) {
        c->pre_gather_valid = false;
        if (t.wait_local_event(c->pre_gather) != 0) return -1;  // aborted and set the error
    }
    return t.wait((hipStream_t)stream) == 0 ? 0 : -1;  // wait() aborted and set the error
}

extern "C" int rt2_render_host_gather(rt2_scene* scene, const rt2_uniforms* u, uint32_t frame_begin,
                                      uint32_t frame_count, rt2_shard sh, rt2_comm* c, int32_t root, float* out_rgba,
                                      uint8_t* out_rgb8) {
    if (!c || !u || root < 0 || root >= c->nranks) {  // seen alike on every rank: nothing issued
        rt2h::set_error("rt2_render_host_gather: bad argument");
        return -1;
    }
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const int H = (int)u->height, W = (int)u->width;
    const bool is_root = c->rank == root;
    // Rank-local failures do not return before the agreement steps: every rank
    // issues the same collectives, then all fail together (rt2_comm_protocol.h).
    std::string aerr;
    if (!scene || frame_count == 0 || W < 1 || H < 0) {
        aerr = "bad argument";
    } else if (sh.nranks != c->nranks || sh.rank != c->rank || rt2_shard_rows(H, sh) < 0) {
        aerr = "shard does not match the communicator";
    } else if (c->comm && !c->aborted) {
        ncclResult_t a = ncclSuccess;
        if (ncclCommGetAsyncError(c->comm, &a) != ncclSuccess || (a != ncclSuccess && a != ncclInProgress))
            aerr = std::string("RCCL asynchronous error: ") + ncclGetErrorString(a);
    }
    const int mr = aerr.empty() ? max_slab_rows(H, sh) : 0, rows = aerr.empty() ? rt2_shard_rows(H, sh) : 0;
    const size_t slab = (size_t)mr * W * 16, whole = aerr.empty() ? (size_t)W * H : 0;
    RcclTransport t{c};
    auto render = [&](bool rgb8, std::string& err) -> int {
        if (c->acc.ensure(slab) || c->res.ensure(slab) || (rgb8 && c->acc8.ensure(slab)) ||
            (is_root && (c->image.ensure(whole * 16) ||
                         (rgb8 && (c->image8.ensure(whole * 16) || c->rgb8.ensure(whole * 3))))) ||
            (is_root && c->nranks > 1 && c->hgathered.ensure(slab * c->nranks)))
            return err = "out of device memory", -1;
        // slab buffers of max_rows rows, zeroed: the rows past this rank's slab
        // are the gather's padding
        if (hipMemsetAsync(c->acc.p, 0, slab, st) != hipSuccess || hipMemsetAsync(c->res.p, 0, slab, st) != hipSuccess ||
            (rgb8 && hipMemsetAsync(c->acc8.p, 0, slab, st) != hipSuccess))
            return err = "hipMemsetAsync failed", -1;
        if (rt2_render(scene, u, frame_begin, frame_count, sh, (float*)c->acc.p, rgb8 ? (uint32_t*)c->acc8.p : nullptr,
                       st) != 0 ||
            rt2_resolve_rgba32f((const float*)c->acc.p, (int64_t)rows * W, frame_count, (float*)c->res.p, st) != 0)
            return err = rt2_last_error(), -1;
        // the render is local: the deadline of agreement 2 starts after it
        // (a render longer than RT2_COMM_TIMEOUT_S aborted a healthy job)
        if (t.wait_local(st) != 0) return err = "the render failed on the device", -1;
        return 0;
    };
    auto gathers = [&](bool rgb8) -> int {
        void* recv = is_root ? (c->nranks == 1 ? c->image.p : c->hgathered.p) : nullptr;
        if (ncclGather(c->res.p, recv, slab, ncclUint8, root, c->comm, st) != ncclSuccess) return -1;
        if (is_root && c->nranks > 1 && rt2_unshard_slabs(c->hgathered.p, mr, W, H, sh, c->image.p, st) != 0)
            return -1;
        if (rgb8) {
            void* recv8 = is_root ? (c->nranks == 1 ? c->image8.p : c->hgathered.p) : nullptr;
            if (ncclGather(c->acc8.p, recv8, slab, ncclUint8, root, c->comm, st) != ncclSuccess) return -1;
            if (is_root && c->nranks > 1 && rt2_unshard_slabs(c->hgathered.p, mr, W, H, sh, c->image8.p, st) != 0)
                return -1;
        }
        return 0;
    };
    // the host waits for the whole sequence under the deadline (a peer that
    // fails inside a gather cannot hang this rank), then the root copies out
    auto finish = [&](bool rgb8, std::string& err) -> int {
        if (is_root && rgb8 && out_rgb8) {
            hipLaunchKernelGGL(rgb8_kernel, dim3((unsigned)((whole + 255) / 256)), dim3(256), 0, st,
                               (const uint4*)c->image8.p, (long long)whole, (float)frame_count, (uint8_t*)c->rgb8.p);
            if (hipGetLastError() != hipSuccess) return err = "the 8-bit resolve failed", -1;
        }
        if (t.wait(st) != 0) return err = "waiting for the gathers failed", -1;
        if (is_root && rgb8 && out_rgb8 && hipMemcpy(out_rgb8, c->rgb8.p, whole * 3, hipMemcpyDeviceToHost) != hipSuccess)
            return err = "the copy of the 8-bit image failed", -1;
        if (is_root && out_rgba && hipMemcpy(out_rgba, c->image.p, whole * 16, hipMemcpyDeviceToHost) != hipSuccess)
            return err = "the copy of the image failed", -1;
        return 0;
    };
    std::string err;
    if (rt2p::render_gather(t, aerr.empty(), aerr, out_rgb8 != nullptr, render, gathers, finish, err) != 0) {
        rt2h::set_error("rt2_render_host_gather: " + err);
        return -1;
    }
    return rt2_comm_check(c);
}
