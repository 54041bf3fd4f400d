// Diagnostic: how much does K1's stage pass (stage_input) slow down while the
// partner wave on its SIMD runs the coupling GEMM (K1t's overlap)?  Uses the
// production device code (kura_kernels.hip) on synthetic records.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I dbs-gym_amd/csrc \
//       -o tools/interfere_bench tools/interfere_bench.hip
// One workgroup per CU (grid 256), 8 waves, N = 1024 (TPW = 4).  Waves 0-3
// ("G") loop over GEMM halves, waves 4-7 ("P") loop over stage passes; each
// wave times its own loop.  Variants strip the GEMM of its alpha loads or of
// its LDS operand reads to find the shared resource.
#include "../dbs-gym_amd/csrc/kura_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

// GEMM half with switches: LOADS (alpha buffer loads; else B from registers),
// LDSR (operand ds_read_b128; else A from registers)
__device__ __forceinline__ void mfma_agpr(floatx16& acc, float a, float b) {
    asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
template <int TPW, bool LOADS, bool LDSR, bool AGPR = false>
__device__ __forceinline__ void gemm_variant(const float* __restrict__ Xs, const float* __restrict__ alpha_sw,
                                             floatx16 (&acc)[TPW]) {
    constexpr int N = TPW * 256;
    constexpr int NK8 = N / 8;
    constexpr int KB0 = 0, KB1 = NK8 / 2;
    constexpr int TSTRIDE = NK8 * 64;
    int lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 3;
    const floatx4* xs4 = reinterpret_cast<const floatx4*>(Xs + (lane >> 5) * XS_HALF + (lane & 31) * 4);
    const float* au = uniform_ptr(alpha_sw);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(au + (size_t)wave * TPW * TSTRIDE * 4), 0, TPW * TSTRIDE * 16, 0x00020000);
    auto ld = [&](int t, int k) -> floatx4 {
        return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + k * 64) * 16,
                                                                                 t * TSTRIDE * 16, 0));
    };
    floatx4 b0[TPW], b1[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        b0[t] = ld(t, KB0);
        b1[t] = ld(t, KB0 + 1);
    }
    floatx4 areg = xs4[0];
#pragma unroll 1
    for (int kb = KB0; kb < KB1; kb += 2) {
        floatx4 a = LDSR ? xs4[kb * (XS_BLOCK / 4)] : areg;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                if (AGPR) mfma_agpr(acc[t], a[s], b0[t][s]);
                else acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b0[t][s], acc[t], 0, 0, 0);
            }
        const int k2 = kb + 2 < KB1 ? kb + 2 : KB1 - 1;
        if (LOADS) {
#pragma unroll
            for (int t = 0; t < TPW; ++t) b0[t] = ld(t, k2);
        }
        __builtin_amdgcn_sched_barrier(0);
        a = LDSR ? xs4[(kb + 1) * (XS_BLOCK / 4)] : areg;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                if (AGPR) mfma_agpr(acc[t], a[s], b1[t][s]);
                else acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b1[t][s], acc[t], 0, 0, 0);
            }
        const int k3 = kb + 3 < KB1 ? kb + 3 : KB1 - 1;
        if (LOADS) {
#pragma unroll
            for (int t = 0; t < TPW; ++t) b1[t] = ld(t, k3);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// mode bit 0: G waves run; bit 1: P waves run; variant: 0 full GEMM, 1 no alpha
// loads, 2 no LDS reads, 3 neither
template <int VAR>
__global__ __launch_bounds__(NTHREADS) void interfere_kernel(int mode, int iters, float* R, const float* alpha,
                                                             float* sink, unsigned long long* cyc) {
    extern __shared__ float Xs[];
    constexpr int TPW = 4, N = 1024;
    const int lane = threadIdx.x & 63, tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (tid < E_WG) {
        s_ctl[tid].h = 0.01f;
        s_kn[tid] = 0.5f;
    }
    for (int i = tid; i < xs_floats(N); i += NTHREADS) Xs[i] = 0.001f * (i & 255);
    __syncthreads();
    unsigned long long t0 = 0, t1 = 0;
    float out = 0.0f;
    const bool g = wv < 4;
    if (g && (mode & 1)) {
        floatx16 acc[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
        for (int it = 0; it < iters; ++it) gemm_variant<TPW, (VAR & 1) == 0, (VAR & 2) == 0, (VAR & 4) != 0>(Xs, alpha, acc);
        asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
        t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int t = 0; t < TPW; ++t) out += acc[t][lane & 15];
    } else if (!g && (mode & 2)) {
        // the P waves write their own columns (as team B would: waves 4-7 own tiles 16..31)
        const Slot ws{__builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(R + (size_t)blockIdx.x * NSLOT * N * 16),
                                                        0, NSLOT * N * 16 * 4, 0x00020000),
                      N, wv * TPW, lane * 16};
        // the pass count of one GEMM half is ~1/4 of a sweep: run a comparable number
        if (mode & 4) __builtin_amdgcn_s_setprio(3);  // the pass wave first at issue arbitration
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
        for (int it = 0; it < iters / 4; ++it) {
            asm volatile("" ::: "memory");  // no hoisting of the record loads out of the loop
            stage_input<TPW>(ws, Xs, 3);
        }
        t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_setprio(0);
    }
    sink[blockIdx.x * NTHREADS + tid] = out;
    if (lane == 0) cyc[blockIdx.x * NWAVES + wv] = t1 - t0;
}

int main() {
    const int grid = 256, iters = 64;
    constexpr int N = 1024;
    float *R, *alpha, *sink;
    unsigned long long* cyc;
    (void)hipMalloc(&R, (size_t)grid * NSLOT * N * 16 * sizeof(float));
    (void)hipMalloc(&alpha, (size_t)N * N * sizeof(float));
    (void)hipMalloc(&sink, grid * NTHREADS * sizeof(float));
    (void)hipMalloc(&cyc, grid * NWAVES * sizeof(unsigned long long));
    (void)hipMemset(R, 0, (size_t)grid * NSLOT * N * 16 * sizeof(float));
    (void)hipMemset(alpha, 0, (size_t)N * N * sizeof(float));
    const size_t lds = xs_floats(N) * sizeof(float);
    (void)hipFuncSetAttribute((const void*)interfere_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)interfere_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)interfere_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)interfere_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)interfere_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)interfere_kernel<7>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    std::vector<unsigned long long> h(grid * NWAVES);
    auto run = [&](int var, int mode, const char* name) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (var) {
                case 0: hipLaunchKernelGGL(interfere_kernel<0>, dim3(grid), dim3(NTHREADS), lds, 0, mode, iters, R, alpha, sink, cyc); break;
                case 1: hipLaunchKernelGGL(interfere_kernel<1>, dim3(grid), dim3(NTHREADS), lds, 0, mode, iters, R, alpha, sink, cyc); break;
                case 2: hipLaunchKernelGGL(interfere_kernel<2>, dim3(grid), dim3(NTHREADS), lds, 0, mode, iters, R, alpha, sink, cyc); break;
                case 3: hipLaunchKernelGGL(interfere_kernel<3>, dim3(grid), dim3(NTHREADS), lds, 0, mode, iters, R, alpha, sink, cyc); break;
                case 4: hipLaunchKernelGGL(interfere_kernel<4>, dim3(grid), dim3(NTHREADS), lds, 0, mode, iters, R, alpha, sink, cyc); break;
                default: hipLaunchKernelGGL(interfere_kernel<7>, dim3(grid), dim3(NTHREADS), lds, 0, mode, iters, R, alpha, sink, cyc); break;
            }
        }
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        std::vector<double> gv, pv;
        for (int b = 0; b < grid; ++b)
            for (int w = 0; w < NWAVES; ++w) {
                const double c = (double)h[b * NWAVES + w];
                if (c > 0) (w < 4 ? gv : pv).push_back(c);
            }
        auto med = [](std::vector<double>& x) {
            if (x.empty()) return 0.0;
            std::sort(x.begin(), x.end());
            return x[x.size() / 2];
        };
        printf("%-44s G: %9.0f cyc/half-GEMM   P: %9.0f cyc/pass\n", name, med(gv) / iters, med(pv) / (iters / 4));
    };
    const char* vn[8] = {"full GEMM", "GEMM without alpha loads", "GEMM without LDS reads", "GEMM without both",
                         "full GEMM, AGPR acc", "", "", "GEMM without both, AGPR acc"};
    run(0, 2, "pass alone");
    for (int v : {0, 4, 3, 7}) {
        char a[96], b[96];
        snprintf(a, sizeof a, "%s alone", vn[v]);
        snprintf(b, sizeof b, "%s + pass", vn[v]);
        run(v, 1, a);
        run(v, 3, b);
        snprintf(b, sizeof b, "%s + pass (pass s_setprio 3)", vn[v]);
        run(v, 7, b);
    }
    return 0;
}
