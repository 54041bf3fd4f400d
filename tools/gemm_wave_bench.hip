// gemm_wave_bench.hip -- diagnostic: how the production coupling GEMM
// (coupling_gemm, kura_kernels.hip) shares a SIMD.  Full grid of 256
// workgroups x 512 threads, N=1024, as in kura_step_kernel.
//   * 8 waves vs waves 0-3 only: does one wave per SIMD saturate the FP32 matrix pipe?
//   * a VALU-only fmod+sincos stream (the element-wise work of a stage) on
//     waves 4-7, alone and beside waves 0-3's MFMAs: what does co-issue cost?
// Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/gemm_wave_bench tools/gemm_wave_bench.hip
//   ./tools/gemm_wave_bench
#include "../dbs-gym_amd/csrc/kura_kernels.hip"

#include <stdio.h>
#include <vector>

// MODE 0: every wave runs the GEMM
// MODE 1: waves 0-3 only (one wave per SIMD)
// MODE 2: waves 0-3 GEMM, waves 4-7 the VALU stream (its cycles reported)
// MODE 3: waves 4-7 the VALU stream alone
template <int MODE>
__global__ __launch_bounds__(NTHREADS) void wave_gemm_kernel(const float* alpha_sw, float* out, int reps) {
    extern __shared__ float Xs[];
    const int N = 1024;
    for (int i = threadIdx.x; i < xs_floats(N); i += NTHREADS) Xs[i] = 0.001f * (float)(i % 97);
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    float sum = 0.0f;
    if (MODE >= 2 && wave >= 4) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        float x = 0.001f * (float)threadIdx.x;
        for (int r = 0; r < reps * 400; ++r) {
            float sn, cs;
            int slow = 0;
            const float th = kdm_fmod2pi_fast(x * 3.0f + 1.0f, &slow);
            kdm_sincosf(th, &sn, &cs);
            x = sn + cs * 0.5f + (float)slow;
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        sum = x;
        if ((threadIdx.x & 63) == 0) out[256 * NTHREADS + blockIdx.x * 8 + wave] = (float)(t1 - t0);
    } else if (MODE == 0 || (MODE != 3 && wave < 4)) {
        const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
        for (int r = 0; r < reps; ++r) {
            floatx16 acc[4];
            coupling_gemm<4>(Xs, alpha_sw, acc);
            for (int t = 0; t < 4; ++t) sum += acc[t][0] + acc[t][15];
        }
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {  // shader clock during the GEMM: s_memtime ticks per 100 MHz s_memrealtime tick
            out[256 * NTHREADS + 256 * 8 + 2 * blockIdx.x] = (float)(c1 - c0);
            out[256 * NTHREADS + 256 * 8 + 2 * blockIdx.x + 1] = (float)(r1 - r0);
        }
    }
    out[blockIdx.x * NTHREADS + threadIdx.x] = sum;
}

template <int MODE>
static void run(const char* name, const float* dA, float* dO) {
    const int N = 1024, nwg = 256, reps = 20;
    const size_t lds = (size_t)xs_floats(N) * 4;
    (void)hipFuncSetAttribute((const void*)wave_gemm_kernel<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL(wave_gemm_kernel<MODE>, dim3(nwg), dim3(NTHREADS), lds, 0, dA, dO, 2);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(wave_gemm_kernel<MODE>, dim3(nwg), dim3(NTHREADS), lds, 0, dA, dO, reps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (MODE >= 2) {
        std::vector<float> h(256 * 8);
        (void)hipMemcpy(h.data(), dO + 256 * NTHREADS, h.size() * 4, hipMemcpyDeviceToHost);
        double c = 0;
        for (int b = 0; b < 256; ++b)
            for (int w = 4; w < 8; ++w) c += h[b * 8 + w];
        printf("%-40s %8.3f ms  VALU stream: %.0f cycles per wave\n", name, ms, c / 1024);
        return;
    }
    std::vector<float> hc(512);
    (void)hipMemcpy(hc.data(), dO + 256 * NTHREADS + 256 * 8, hc.size() * 4, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int b = 0; b < 256; ++b) cyc += hc[2 * b], rt += hc[2 * b + 1];
    const int waves = MODE == 0 ? 8 : 4;
    printf("%-40s shader clock during the GEMM: %.2f GHz\n", name, cyc / rt * 0.1);
    // per active wave per rep: 32 rows x (4 tiles x 32 cols) x N x 2 flop
    const double flop = (double)nwg * waves * reps * 32.0 * 128.0 * N * 2.0;
    printf("%-40s %8.3f ms  %6.1f TFLOP/s\n", name, ms, flop / (ms * 1e-3) / 1e12);
}

int main() {
    const int N = 1024;
    std::vector<float> h((size_t)N * N);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.35f + 0.65f * (float)((i * 2654435761u) % 1000) / 1000.0f;
    float *dA, *dO;
    (void)hipMalloc(&dA, h.size() * 4);
    (void)hipMalloc(&dO, 256 * NTHREADS * 4 + 256 * 8 * 4 + 512 * 4);
    (void)hipMemcpy(dA, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    run<0>("8 waves, GEMM", dA, dO);
    run<1>("waves 0-3 only, GEMM", dA, dO);
    run<2>("waves 0-3 GEMM + waves 4-7 VALU stream", dA, dO);
    run<3>("waves 4-7 VALU stream alone", dA, dO);
    return 0;
}
