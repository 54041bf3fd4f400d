// Microbenchmark 2: which instruction kinds of a wave are slowed while the
// other wave on its SIMD streams v_mfma_f32_32x32x2_f32?  (K1t diagnosis,
// DESIGN.md section 5; profiles/r03_overlap_microbench2.txt.)
//   hipcc --offload-arch=gfx950 -O3 -o tools/overlap_bench2 tools/overlap_bench2.hip
// 256 workgroups x 8 waves; waves 0-3 stream MFMAs (4 accumulators) when
// `mfma` is set, waves 4-7 run probe KIND; each wave times its own loop.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
#define ITERS 2048

template <int KIND>
__global__ __launch_bounds__(512) void probe_kernel(int mfma, float* buf, float* sink, unsigned long long* cyc) {
    __shared__ float lds[8 * 64 * 4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long t0 = 0, t1 = 0;
    float out = 0.0f;
    __syncthreads();
    if (wave < 4) {
        if (mfma) {
            floatx16 acc[4];
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
            const float a = lane * 1e-3f, b = 1.0f;
            t0 = __builtin_amdgcn_s_memtime();
            if (mfma == 1) {
#pragma unroll 1
                for (int it = 0; it < ITERS * 8; ++it)
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
            } else if (mfma == 2) {  // 32 MFMAs per loop iteration
#pragma unroll 1
                for (int it = 0; it < ITERS; ++it)
#pragma unroll
                    for (int r = 0; r < 8; ++r)
#pragma unroll
                        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
            } else {  // 32 per iteration, accumulators in AGPRs
#pragma unroll 1
                for (int it = 0; it < ITERS; ++it)
#pragma unroll
                    for (int r = 0; r < 8; ++r)
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc[t]) : "v"(a), "v"(b));
                asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
            }
            t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
            for (int t = 0; t < 4; ++t) out += acc[t][lane & 15];
        }
    } else {
        float v = lane * 1e-3f, w = 1.0f + lane;
        float* lp = lds + (wave * 64 + lane) * 4;
        float* gp = buf + ((size_t)blockIdx.x * 512 + threadIdx.x) * 4;
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
        for (int it = 0; it < ITERS; ++it) {
            if (KIND == 0) {  // 16 independent fma chains
                float x[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) x[k] = v + k;
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int k = 0; k < 16; ++k) x[k] = __builtin_fmaf(x[k], 1.0001f, 0.5f);
#pragma unroll
                for (int k = 0; k < 16; ++k) v += x[k] * 1e-9f;
            } else if (KIND == 1) {  // one dependent chain of 64 fma
#pragma unroll
                for (int k = 0; k < 64; ++k) v = __builtin_fmaf(v, 1.0001f, 0.5f);
            } else if (KIND == 2) {  // LDS write + dependent read, 8 per iteration
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    lp[k & 3] = v;
                    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
                    v = lp[(k + 1) & 3] + 1.0f;
                }
            } else if (KIND == 3) {  // global load + wait, 4 per iteration
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v += __builtin_nontemporal_load(gp + (k & 3));
                    asm volatile("" ::: "memory");
                }
            } else if (KIND == 4) {  // compare + select chain (VCC)
#pragma unroll
                for (int k = 0; k < 32; ++k) v = v > w ? v - w : v + 0.25f;
            } else if (KIND == 5) {  // v_readlane / SALU mix
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int s = __builtin_amdgcn_readfirstlane(__float_as_int(v));
                    v = v + __int_as_float((s & 0x3f) | 0x3f800000);
                }
            } else if (KIND == 7) {  // overlap_bench's VALU loop: 16 chains, one fma each per iteration
                static_assert(true, "");
                // (kept in registers across iterations via the asm barrier below)
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    v = __builtin_fmaf(v, 1.0001f, 0.5f);
                    w = __builtin_fmaf(w, 0.9999f, 0.25f);
                }
            } else if (KIND == 6) {  // f32 trunc/rint/cvt mix (fmod / sincos reduction)
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const float q = truncf(v * 0.159f);
                    const float j = rintf(v * 0.63f);
                    v = __builtin_fmaf(-q, 6.28f, v) + (float)(((int)j) & 3);
                }
            }
        }
        t1 = __builtin_amdgcn_s_memtime();
        out = v + w;
    }
    sink[blockIdx.x * 512 + threadIdx.x] = out;
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

int main() {
    const int grid = 256;
    float *sink, *buf;
    unsigned long long* cyc;
    (void)hipMalloc(&sink, grid * 512 * sizeof(float));
    (void)hipMalloc(&buf, grid * 512 * 4 * sizeof(float));
    (void)hipMemset(buf, 0, grid * 512 * 4 * sizeof(float));
    (void)hipMalloc(&cyc, grid * 8 * sizeof(unsigned long long));
    std::vector<unsigned long long> h(grid * 8);
    const char* names[8] = {"16 indep fma chains x4", "1 dependent fma chain x64", "LDS write+read x8",
                            "global load x4 (L2-hot)", "cmp+select chain x32", "readfirstlane+add x16",
                            "trunc/rint/cvt mix x16", "2 chains x16 fma"};
    for (int kind = 0; kind < 8; ++kind) {
        double res[4];
        for (int m = 0; m < 4; ++m) {
            for (int rep = 0; rep < 2; ++rep) {
                switch (kind) {
                    case 0: hipLaunchKernelGGL(probe_kernel<0>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                    case 1: hipLaunchKernelGGL(probe_kernel<1>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                    case 2: hipLaunchKernelGGL(probe_kernel<2>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                    case 3: hipLaunchKernelGGL(probe_kernel<3>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                    case 4: hipLaunchKernelGGL(probe_kernel<4>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                    case 5: hipLaunchKernelGGL(probe_kernel<5>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                    case 6: hipLaunchKernelGGL(probe_kernel<6>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                    default: hipLaunchKernelGGL(probe_kernel<7>, dim3(grid), dim3(512), 0, 0, m, buf, sink, cyc); break;
                }
            }
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            std::vector<double> p;
            for (int b = 0; b < grid; ++b)
                for (int w = 4; w < 8; ++w) p.push_back((double)h[b * 8 + w]);
            std::sort(p.begin(), p.end());
            res[m] = p[p.size() / 2] / ITERS;
        }
        printf("%-28s alone %8.1f cyc/iter | beside MFMA: 4/iter %8.1f (x%.2f)  32/iter %8.1f (x%.2f)  32/iter AGPR %8.1f (x%.2f)\n",
               names[kind], res[0], res[1], res[1] / res[0], res[2], res[2] / res[0], res[3], res[3] / res[0]);
    }
    return 0;
}
