// Micro-probe (diagnostic, not part of the product): can one SIMD overlap the
// k16 sweep's matrix products with the reduction VALU of other waves?
// Each wave loops over "groups" of the render kernel's shape — per 32-ray
// block 6 v_mfma_f32_32x32x16_f16 | 16 v_max3_i32 | 2 MFMA | 16 v_max3_i32 +
// 8 v_min3_i32 — on register operands (no memory traffic), in four modes:
//   0 dep   : the kernel's order (each block's VALU reads that block's products)
//   1 mfma  : the 16 products only (two accumulation chains)
//   2 valu  : the 80 VALU only
//   3 indep : products (mode 1) and VALU (mode 2) in the same wave, no
//             dependency between them (the compiler interleaves them)
//   4 split : odd workgroups run mode 1, even ones mode 2 (each SIMD holds
//             matrix-only and VALU-only waves: do they overlap?)
// at 1..4 waves per SIMD (occupancy set by the grid: one 256-thread workgroup
// of 4 waves per CU-slot, W slots per CU).  Prints SIMD clocks per wave-group.
// Build: hipcc -O3 --offload-arch=gfx950 -o overlap_probe overlap_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

#define MF(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0)
#define FENCE() __builtin_amdgcn_sched_barrier(0)

#define TOUCH(x) asm volatile("" : "+v"(x))  // the value "changes" every iteration: no hoisting

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void probe(const h8* in, int iters, int* sink, unsigned long long* clk) {
    const int l = threadIdx.x & 63;
    h8 a0 = in[l], a1 = in[64 + l], y1 = in[128 + l];
    h8 b[7];
#pragma unroll
    for (int k = 0; k < 7; k++) b[k] = in[192 + 64 * k + l];
    const f16v zero = {};
    // VALU operands (modes 2-4): products of the inputs, computed once
    f16v pU = MF(a0, b[0], zero), pV = MF(a0, b[2], zero);
    int tmin = 0x7fffffff, acc = 0;
    f16v cU = zero, cV = zero;  // mode 1 chains
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int R = 0; R < 2; R++) {
            if constexpr (MODE == 0) {
                f16v U = MF(a0, b[0], zero), V = MF(a0, b[2], zero), X = MF(a0, b[4], zero);
                U = MF(a1, b[1], U);
                V = MF(a1, b[3], V);
                X = MF(a1, b[5], X);
                FENCE();
                int t3[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    t3[i] = max(max(__float_as_int(U[i]), __float_as_int(V[i])), __float_as_int(X[i]));
                FENCE();
                const f16v T = MF(a1, b[6], zero), Y = MF(y1, b[6], zero);
                FENCE();
#pragma unroll
                for (int i = 0; i < 16; i++) tmin = min(tmin, max(max(t3[i], __float_as_int(T[i])), __float_as_int(Y[i])));
            } else if constexpr (MODE == 1) {
                cU = MF(a0, b[0], cU);
                cV = MF(a0, b[2], cV);
                cU = MF(a0, b[4], cU);
                cV = MF(a1, b[1], cV);
                cU = MF(a1, b[3], cU);
                cV = MF(a1, b[5], cV);
                cU = MF(a1, b[6], cU);
                cV = MF(y1, b[6], cV);
            } else {
                const bool do_mfma = MODE == 3 || (MODE == 4 && (blockIdx.x & 1));
                const bool do_valu = MODE == 2 || MODE == 3 || (MODE == 4 && !(blockIdx.x & 1));
                if (do_mfma) {
                    cU = MF(a0, b[0], cU);
                    cV = MF(a0, b[2], cV);
                    cU = MF(a0, b[4], cU);
                    cV = MF(a1, b[1], cV);
                    cU = MF(a1, b[3], cU);
                    cV = MF(a1, b[5], cV);
                    cU = MF(a1, b[6], cU);
                    cV = MF(y1, b[6], cV);
                }
                if (do_valu) {
                    TOUCH(pU);
                    TOUCH(pV);
                    int t3[16];
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        t3[i] = max(max(__float_as_int(pU[i]), __float_as_int(pV[i])), __float_as_int(pV[15 - i]));
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        tmin = min(tmin, max(max(t3[i], __float_as_int(pU[15 - i])), __float_as_int(pV[(i + 3) & 15])));
                }
            }
        }
        acc += __builtin_amdgcn_readfirstlane(tmin) & 1;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if constexpr (MODE != 0 && MODE != 2) tmin ^= __float_as_int(cU[0]) ^ __float_as_int(cV[3]);
    if (tmin == 0x12345 || acc == -7) sink[0] = tmin;
    if (l == 0) clk[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
static double run(int slots, int iters, const h8* d_in, int* d_sink, unsigned long long* d_clk, float* ms) {
    const int blocks = 256 * slots;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, d_in, iters, d_sink, d_clk);  // warm
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, d_in, iters, d_sink, d_clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(ms, e0, e1);
    std::vector<unsigned long long> c(blocks * 4);
    hipMemcpy(c.data(), d_clk, c.size() * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : c) s += (double)v;
    return s / c.size() / iters;  // wave clocks per group
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    std::vector<_Float16> h(8 * 64 * 10);
    srand(1);
    for (auto& x : h) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 2.0f);
    h8* d_in;
    int* d_sink;
    unsigned long long* d_clk;
    hipMalloc(&d_in, h.size() * 2);
    hipMalloc(&d_sink, 4);
    hipMalloc(&d_clk, 256 * 8 * 4 * 8);
    hipMemcpy(d_in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const char* names[5] = {"dep", "mfma", "valu", "indep", "split"};
    for (int slots = 1; slots <= 4; slots++) {
        for (int mode = 0; mode < 5; mode++) {
            float ms = 0;
            double wc = mode == 0   ? run<0>(slots, iters, d_in, d_sink, d_clk, &ms)
                        : mode == 1 ? run<1>(slots, iters, d_in, d_sink, d_clk, &ms)
                        : mode == 2 ? run<2>(slots, iters, d_in, d_sink, d_clk, &ms)
                        : mode == 3 ? run<3>(slots, iters, d_in, d_sink, d_clk, &ms)
                                    : run<4>(slots, iters, d_in, d_sink, d_clk, &ms);
            // SIMD clocks per wave-group: the wave's clocks per group / waves sharing the SIMD
            const double groups = 256.0 * slots * 4 * iters;
            printf("{\"waves_per_simd\": %d, \"mode\": \"%s\", \"wave_clocks_per_group\": %.1f, "
                   "\"simd_clocks_per_wave_group\": %.1f, \"kernel_ms\": %.3f, \"ns_per_wave_group_per_simd\": %.3f}\n",
                   slots, names[mode], wc, wc / slots, ms, ms * 1e6 / (groups / 1024.0));
            fflush(stdout);
        }
    }
    return 0;
}
