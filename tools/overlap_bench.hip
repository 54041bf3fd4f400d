// Microbenchmark: does f32 VALU work overlap with v_mfma_f32_32x32x2_f32 on
// one SIMD?  (K1t design question)
//   hipcc --offload-arch=gfx950 -O3 -o tools/overlap_bench tools/overlap_bench.hip
// One workgroup per CU (grid 256), 8 waves.  Waves 0-3 run an MFMA loop
// (TW independent accumulators, back-to-back issue), waves 4-7 a VALU loop
// (independent v_fma_f32 chains); mode selects which groups run.  Every wave
// times its own loop with s_memtime; the host prints the median per group.
// mode 0: MFMA only; 1: VALU only; 2: both; 3: one wave per SIMD (waves 0-3)
// with VALU interleaved into its own MFMA stream (NV v_fma per MFMA).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

#define ITERS 4096
#define TW 4

template <int NV>
__global__ __launch_bounds__(512) void overlap_kernel(int mode, float* sink, unsigned long long* cyc, int* simd) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float a0 = lane * 1e-3f, b0 = 1.0f + lane * 1e-4f;
    unsigned long long t0 = 0, t1 = 0;
    float out = 0.0f;
    const bool mfma_wave = wave < 4;
    // 4: MFMA wave + packed-f32 (v_pk_fma_f32) wave; 5: packed-f32 waves alone
    const bool run = mode == 0 ? mfma_wave : mode == 1 ? !mfma_wave : mode == 2 || mode == 4 ? true
                     : mode == 5 ? !mfma_wave : mfma_wave;
    __syncthreads();
    if (run && mfma_wave) {
        floatx16 acc[TW];
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = a0 + k;
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
            for (int t = 0; t < TW; ++t) {
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[t], 0, 0, 0);
                // NV VALU ops beside each MFMA (mode 3 instantiations only)
#pragma unroll
                for (int k = 0; k < NV; ++k) v[k & 7] = __builtin_fmaf(v[k & 7], 1.0001f, 0.5f);
            }
        }
        t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) out += acc[t][r];
#pragma unroll
        for (int k = 0; k < 8; ++k) out += v[k];
    } else if (run && (mode == 4 || mode == 5)) {
        floatx2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = floatx2{a0 + k, a0 - k};
        const floatx2 c1 = {1.0001f, 1.0002f}, c2 = {0.5f, 0.25f};
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = __builtin_elementwise_fma(v[k], c1, c2);
        }
        t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int k = 0; k < 8; ++k) out += v[k][0] + v[k][1];
    } else if (run) {
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = a0 + k;
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = __builtin_fmaf(v[k], 1.0001f, 0.5f);
        }
        t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int k = 0; k < 16; ++k) out += v[k];
    }
    sink[blockIdx.x * 512 + threadIdx.x] = out;
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = run ? t1 - t0 : 0;
    if (lane == 0) simd[blockIdx.x * 8 + wave] = (__builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11)) >> 4) & 3;
}

int main() {
    const int grid = 256;
    float* sink;
    unsigned long long* cyc;
    hipMalloc(&sink, grid * 512 * sizeof(float));
    hipMalloc(&cyc, grid * 8 * sizeof(unsigned long long));
    int* simd;
    hipMalloc(&simd, grid * 8 * sizeof(int));
    std::vector<int> hs(grid * 8);
    std::vector<unsigned long long> h(grid * 8);
    auto run = [&](int mode, int nv, const char* name) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (nv) {
                case 0: hipLaunchKernelGGL(overlap_kernel<0>, dim3(grid), dim3(512), 0, 0, mode, sink, cyc, simd); break;
                case 2: hipLaunchKernelGGL(overlap_kernel<2>, dim3(grid), dim3(512), 0, 0, mode, sink, cyc, simd); break;
                case 4: hipLaunchKernelGGL(overlap_kernel<4>, dim3(grid), dim3(512), 0, 0, mode, sink, cyc, simd); break;
                case 8: hipLaunchKernelGGL(overlap_kernel<8>, dim3(grid), dim3(512), 0, 0, mode, sink, cyc, simd); break;
                case 12: hipLaunchKernelGGL(overlap_kernel<12>, dim3(grid), dim3(512), 0, 0, mode, sink, cyc, simd); break;
                default: hipLaunchKernelGGL(overlap_kernel<16>, dim3(grid), dim3(512), 0, 0, mode, sink, cyc, simd); break;
            }
        }
        hipDeviceSynchronize();
        hipMemcpy(h.data(), cyc, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::vector<double> m, v;
        for (int b = 0; b < grid; ++b)
            for (int w = 0; w < 8; ++w) {
                const double c = (double)h[b * 8 + w];
                if (c == 0) continue;
                (w < 4 ? m : v).push_back(c);
            }
        auto med = [](std::vector<double>& x) {
            if (x.empty()) return 0.0;
            std::sort(x.begin(), x.end());
            return x[x.size() / 2];
        };
        const double mm = med(m), vv = med(v);
        hipMemcpy(hs.data(), simd, hs.size() * sizeof(int), hipMemcpyDeviceToHost);
        int same = 0;  // workgroups in which wave w and wave w+4 share a SIMD for every w
        for (int b = 0; b < grid; ++b) {
            bool ok = true;
            for (int w = 0; w < 4; ++w) ok = ok && hs[b * 8 + w] == hs[b * 8 + w + 4];
            same += ok;
        }
        if (mode == 2) printf("  (w, w+4 on one SIMD in %d of %d workgroups; wg0 simds %d%d%d%d %d%d%d%d)\n", same, grid,
                              hs[0], hs[1], hs[2], hs[3], hs[4], hs[5], hs[6], hs[7]);
        // per MFMA (ITERS*TW of them) and per VALU fma (ITERS*16)
        printf("%-34s mfma waves: %10.0f cyc (%6.1f cyc/mfma)   valu waves: %10.0f cyc (%5.2f cyc/fma)\n", name, mm,
               mm / (ITERS * TW), vv, vv / (ITERS * 16));
    };
    run(0, 0, "MFMA only (1 wave/SIMD)");
    run(1, 0, "VALU only (1 wave/SIMD)");
    run(2, 0, "MFMA wave + VALU wave per SIMD");
    run(5, 0, "pk_fma only (1 wave/SIMD; cyc/2 fma)");
    run(4, 0, "MFMA wave + pk_fma wave per SIMD");
    for (int nv : {0, 2, 4, 8, 12, 16}) {
        char name[64];
        snprintf(name, sizeof name, "one wave, %d fma per MFMA", nv);
        run(3, nv, name);
    }
    return 0;
}
