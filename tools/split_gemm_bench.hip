// split_gemm_bench.hip -- diagnostic for DESIGN.md section 9: can the coupling
// GEMM (32 operand rows x N=1024 x N, 16 envs per workgroup, one workgroup per
// CU, 8 waves x 4 column tiles) run faster as three-way bf16 splits on
// v_mfma_f32_32x32x16_bf16, and where do its B fragments come from?
//   f32_stream   : production form -- fp32 32x32x2 MFMAs, alpha fragments
//                  streamed from L2 by raw buffer loads (the baseline)
//   f32_table    : same MFMAs, B gathered from the grid-displacement table in
//                  LDS (alpha is an exact function of |dx|,|dy|,|dz|)
//   split_stream : x and alpha as 3 bf16 parts, six 32x32x16 bf16 MFMAs per
//                  16-deep k-block; alpha parts pre-split in global memory
//   split_table  : as split_stream, alpha parts gathered from the LDS table
//   split_noload : as split_stream with B fixed in registers (MFMA + x-split
//                  ceiling)
// f32_table == f32_stream and split_table == split_stream bit for bit (same
// operands, same order); the split forms are compared with the exact sum.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/split_gemm_bench tools/split_gemm_bench.hip
//   ./tools/split_gemm_bench [reps] [dump.bin] [trace.bin]
// dump.bin: split_stream's outputs of workgroup 0 (512 threads x 4 tiles x 16
// floats, the raw accumulator layout) for tools/split_gemm_check.py, which
// recomputes them with the oracle's exact bf16 MFMA model
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

constexpr int N = 1024, NKB = N / 16, CT = N / 32, TPW = 4, NW = 8, NT = NW * 64;
constexpr int GX = 16, GY = 8, GZ = 8;     // neuron grid: flat n = (z*GX + x)*GY + y
constexpr int NCLS = GX * GZ;              // (|dx|, |dz|) classes; |dy| runs along a mirrored row
constexpr int XS_BYTES = N * 32 * 4;       // operand, fragment layout [kb][j][lane] float4

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float operand(int row, int k, int w) {
    unsigned h = (unsigned)(row * N + k) * 2654435761u + (unsigned)w * 40503u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    return (float)(h & 0xffff) / 32768.0f - 1.0f;
}

__device__ __forceinline__ int lane_id() {
    int lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    return lane;
}

// x = h1 + h2 + h3 exactly for |x| in the normal range (each residual is exact in f32)
__device__ __forceinline__ void split8(f32x4 lo, f32x4 hi, bf16x8& h1, bf16x8& h2, bf16x8& h3) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float x = i < 4 ? lo[i] : hi[i - 4];
        const __bf16 a = (__bf16)x;
        const float r1 = x - (float)a;
        const __bf16 b = (__bf16)r1;
        const float r2 = r1 - (float)b;
        h1[i] = a;
        h2[i] = b;
        h3[i] = (__bf16)r2;
    }
}

__device__ __forceinline__ void mfma6(f32x16& acc, const bf16x8& x1, const bf16x8& x2, const bf16x8& x3,
                                      const bf16x8& a1, const bf16x8& a2, const bf16x8& a3) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1, a1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1, a2, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x2, a1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1, a3, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x2, a2, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x3, a1, acc, 0, 0, 0);
}

// V: 0 f32_stream, 1 f32_table, 2 split_stream, 3 split_table, 4 split_noload
// gA: fp32 alpha [ct][kb][j][lane] float4; gS: split alpha [ct][kb][p][lane] 8 x bf16;
// gT: mirrored table rows, fp32 [cls][16] (V1) or u32x2 {p1 | p2 << 16, p3} [cls][16] (V3)
template <int V>
__global__ __launch_bounds__(NT) void gemm(const float* __restrict__ gA, const uint16_t* __restrict__ gS,
                                           const void* __restrict__ gT, float* __restrict__ out, int reps) {
    extern __shared__ float4 lds[];
    f32x4* xs = reinterpret_cast<f32x4*>(lds);
    const int tid = threadIdx.x;
    for (int q = tid; q < NKB * 2 * 64; q += NT) {   // q = (kb*2 + j)*64 + lane
        const int l = q & 63, j = (q >> 6) & 1, kb = q >> 7;
        f32x4 v;
        for (int c = 0; c < 4; ++c) v[c] = operand(l & 31, kb * 16 + 8 * (l >> 5) + 4 * j + c, blockIdx.x);
        xs[q] = v;
    }
    float* tf = reinterpret_cast<float*>(lds) + XS_BYTES / 4;           // V1 table
    u32x2* tq = reinterpret_cast<u32x2*>(reinterpret_cast<char*>(lds) + XS_BYTES);   // V3 table
    if (V == 1)
        for (int q = tid; q < NCLS * 16; q += NT) tf[q] = reinterpret_cast<const float*>(gT)[q];
    if (V == 3)
        for (int q = tid; q < NCLS * 16; q += NT) tq[q] = reinterpret_cast<const u32x2*>(gT)[q];
    __syncthreads();
    const int lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // table addressing: column c = ct*32 + lane%32 -> y_c = lane%8, line L_c = ct*4 + (lane%32)/8;
    // k = kb*16 + 8*(lane/32) + i -> y_k = i, line L_k = kb*2 + lane/32; x = L%16, z = L/16
    int xc[TPW], zc[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int lc = (wave * TPW + t) * 4 + ((lane & 31) >> 3);
        xc[t] = lc % GX;
        zc[t] = lc / GX;
    }
    const int yoff = 7 - (lane & 7);   // row entry of i = 0 (row[j] = T[|j - 7|])
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(gA + (size_t)wave * TPW * NKB * 2 * 64 * 4), 0, TPW * NKB * 2 * 64 * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(gS + (size_t)wave * TPW * NKB * 3 * 64 * 8), 0, TPW * NKB * 3 * 64 * 16, 0x00020000);
    f32x16 acc[TPW];
    for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
        if (V == 0) {
            auto ld = [&](int t, int kb, int j) -> f32x4 {
                return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     ra, ((kb * 2 + j) * 64 + lane) * 16, t * NKB * 2 * 64 * 16, 0));
            };
            f32x4 b0[TPW], b1[TPW];
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                b0[t] = ld(t, 0, 0);
                b1[t] = ld(t, 0, 1);
            }
#pragma unroll 1
            for (int kb = 0; kb < NKB; ++kb) {
                const int kn = kb + 1 < NKB ? kb + 1 : NKB - 1;
                f32x4 a = xs[(kb * 2 + 0) * 64 + lane];
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < TPW; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b0[t][s], acc[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < TPW; ++t) b0[t] = ld(t, kn, 0);
                __builtin_amdgcn_sched_barrier(0);
                a = xs[(kb * 2 + 1) * 64 + lane];
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int t = 0; t < TPW; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b1[t][s], acc[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < TPW; ++t) b1[t] = ld(t, kn, 1);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if (V == 1) {
#pragma unroll 1
            for (int kb = 0; kb < NKB; ++kb) {
                const int lk = kb * 2 + (lane >> 5), xk = lk % GX, zk = lk / GX;
                const f32x4 a0 = xs[(kb * 2 + 0) * 64 + lane], a1 = xs[(kb * 2 + 1) * 64 + lane];
                float b[TPW][8];
#pragma unroll
                for (int t = 0; t < TPW; ++t) {
                    const int base = (__builtin_abs(zk - zc[t]) * GX +
                                      __builtin_abs(xk - xc[t])) * 16 + yoff;
#pragma unroll
                    for (int i = 0; i < 8; ++i) b[t][i] = tf[base + i];
                }
#pragma unroll
                for (int s = 0; s < 8; ++s)
#pragma unroll
                    for (int t = 0; t < TPW; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(s < 4 ? a0[s] : a1[s - 4], b[t][s], acc[t], 0,
                                                                       0, 0);
            }
        } else {
            bf16x8 c1, c2, c3;
            if (V == 4) {
                const u32x4 w = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsp, lane * 16, 0, 0));
                c1 = __builtin_bit_cast(bf16x8, w);
                c2 = __builtin_bit_cast(bf16x8, w ^ 0x00010001u);
                c3 = __builtin_bit_cast(bf16x8, w ^ 0x00020002u);
            }
            auto lds_split = [&](int t, int kb, bf16x8& p1, bf16x8& p2, bf16x8& p3) {
                const int lk = kb * 2 + (lane >> 5), xk = lk % GX, zk = lk / GX;
                const int base = (__builtin_abs(zk - zc[t]) * GX +
                                  __builtin_abs(xk - xc[t])) * 16 + yoff;
                u32x2 e[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) e[i] = tq[base + i];
                u32x4 w1, w2, w3;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    w1[q] = __builtin_amdgcn_perm(e[2 * q + 1].x, e[2 * q].x, 0x05040100u);
                    w2[q] = __builtin_amdgcn_perm(e[2 * q + 1].x, e[2 * q].x, 0x07060302u);
                    w3[q] = __builtin_amdgcn_perm(e[2 * q + 1].y, e[2 * q].y, 0x05040100u);
                }
                p1 = __builtin_bit_cast(bf16x8, w1);
                p2 = __builtin_bit_cast(bf16x8, w2);
                p3 = __builtin_bit_cast(bf16x8, w3);
            };
            auto gld = [&](int t, int kb, int p) -> bf16x8 {
                return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rsp, ((kb * 3 + p) * 64 + lane) * 16, t * NKB * 3 * 64 * 16, 0));
            };
            bf16x8 n1[TPW], n2[TPW], n3[TPW];
            if (V == 2) {
#pragma unroll
                for (int t = 0; t < TPW; ++t) {
                    n1[t] = gld(t, 0, 0);
                    n2[t] = gld(t, 0, 1);
                    n3[t] = gld(t, 0, 2);
                }
            }
#pragma unroll 1
            for (int kb = 0; kb < NKB; ++kb) {
                bf16x8 x1, x2, x3;
                split8(xs[(kb * 2 + 0) * 64 + lane], xs[(kb * 2 + 1) * 64 + lane], x1, x2, x3);
                if (V == 2) {
                    const int kn = kb + 1 < NKB ? kb + 1 : NKB - 1;
                    bf16x8 p1[TPW], p2[TPW], p3[TPW];
#pragma unroll
                    for (int t = 0; t < TPW; ++t) {
                        p1[t] = n1[t];
                        p2[t] = n2[t];
                        p3[t] = n3[t];
                        n1[t] = gld(t, kn, 0);
                        n2[t] = gld(t, kn, 1);
                        n3[t] = gld(t, kn, 2);
                    }
#pragma unroll
                    for (int t = 0; t < TPW; ++t) mfma6(acc[t], x1, x2, x3, p1[t], p2[t], p3[t]);
                } else if (V == 3) {
                    bf16x8 p1[TPW], p2[TPW], p3[TPW];
#pragma unroll
                    for (int t = 0; t < TPW; ++t) lds_split(t, kb, p1[t], p2[t], p3[t]);
#pragma unroll
                    for (int t = 0; t < TPW; ++t) mfma6(acc[t], x1, x2, x3, p1[t], p2[t], p3[t]);
                } else {
#pragma unroll
                    for (int t = 0; t < TPW; ++t) mfma6(acc[t], x1, x2, x3, c1, c2, c3);
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) out[((size_t)(blockIdx.x * NT + tid) * TPW + t) * 16 + r] = acc[t][r];
}

// Trace of one 32x32 tile's split chain (column tile 0, workgroup 0's
// operand): the accumulator after every one of the NKB*6 MFMAs, so a model
// mismatch can be pinned to the first MFMA (and its A, B, C) that departs.
__global__ __launch_bounds__(64) void trace(const uint16_t* __restrict__ gS, float* __restrict__ tr) {
    const int lane = threadIdx.x;
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    const u32x4* sp = reinterpret_cast<const u32x4*>(gS);   // tile 0: [kb][p][lane] 16 B
    for (int kb = 0; kb < NKB; ++kb) {
        f32x4 lo, hi;
        for (int c = 0; c < 4; ++c) {
            lo[c] = operand(lane & 31, kb * 16 + 8 * (lane >> 5) + c, 0);
            hi[c] = operand(lane & 31, kb * 16 + 8 * (lane >> 5) + 4 + c, 0);
        }
        bf16x8 x[3], a[3];
        split8(lo, hi, x[0], x[1], x[2]);
        for (int p = 0; p < 3; ++p) a[p] = __builtin_bit_cast(bf16x8, sp[(kb * 3 + p) * 64 + lane]);
        const int pi[6] = {0, 0, 1, 0, 1, 2}, pj[6] = {0, 1, 0, 2, 1, 0};
        for (int q = 0; q < 6; ++q) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[pi[q]], a[pj[q]], acc, 0, 0, 0);
            for (int r = 0; r < 16; ++r) tr[((size_t)(kb * 6 + q) * 64 + lane) * 16 + r] = acc[r];
        }
    }
}

// ---------------------------------------------------------------- host ----
static uint16_t bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static float bf2f(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static float h_operand(int row, int k, int w) {
    unsigned h = (unsigned)(row * N + k) * 2654435761u + (unsigned)w * 40503u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    return (float)(h & 0xffff) / 32768.0f - 1.0f;
}

template <int V>
static double run(const float* dA, const uint16_t* dS, const void* dT, float* dO, int nwg, int reps) {
    const size_t lds = XS_BYTES + (V == 1 ? NCLS * 16 * 4 : V == 3 ? NCLS * 16 * 8 : 0);
    hipFuncSetAttribute((const void*)gemm<V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(gemm<V>, dim3(nwg), dim3(NT), lds, 0, dA, dS, dT, dO, 1);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(gemm<V>, dim3(nwg), dim3(NT), lds, 0, dA, dS, dT, dO, reps);
    hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return -1.0;
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return (double)nwg * reps * 2.0 * 32 * N * N / (ms * 1e-3) / 1e12;   // fp32-equivalent TFLOP/s
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    const int nwg = 256;
    // alpha = f32(cos(0.1 |g_i - g_j|)) from its displacement table
    std::vector<float> T((size_t)GX * GY * GZ);
    for (int dz = 0; dz < GZ; ++dz)
        for (int dx = 0; dx < GX; ++dx)
            for (int dy = 0; dy < GY; ++dy)
                T[(dz * GX + dx) * GY + dy] = (float)cos(0.1 * sqrt((double)(dx * dx + dy * dy + dz * dz)));
    auto gxyz = [](int n, int& x, int& y, int& z) {
        y = n % GY;
        x = (n / GY) % GX;
        z = n / (GX * GY);
    };
    std::vector<float> alpha((size_t)N * N);
    for (int k = 0; k < N; ++k)
        for (int c = 0; c < N; ++c) {
            int xk, yk, zk, xc, yc, zc;
            gxyz(k, xk, yk, zk);
            gxyz(c, xc, yc, zc);
            alpha[(size_t)k * N + c] = T[(abs(zk - zc) * GX + abs(xk - xc)) * GY + abs(yk - yc)];
        }
    std::vector<float> hA((size_t)N * N);
    std::vector<uint16_t> hS((size_t)N * N * 3);
    for (int ct = 0; ct < CT; ++ct)
        for (int kb = 0; kb < NKB; ++kb)
            for (int l = 0; l < 64; ++l)
                for (int i = 0; i < 8; ++i) {
                    const int k = kb * 16 + 8 * (l >> 5) + i, c = ct * 32 + (l & 31);
                    const float a = alpha[(size_t)k * N + c];
                    hA[(((size_t)(ct * NKB + kb) * 2 + (i >> 2)) * 64 + l) * 4 + (i & 3)] = a;
                    const uint16_t h1 = bf16_rne(a);
                    const float r1 = a - bf2f(h1);
                    const uint16_t h2 = bf16_rne(r1);
                    const uint16_t h3 = bf16_rne(r1 - bf2f(h2));
                    const uint16_t hp[3] = {h1, h2, h3};
                    for (int p = 0; p < 3; ++p) hS[(((size_t)(ct * NKB + kb) * 3 + p) * 64 + l) * 8 + i] = hp[p];
                }
    std::vector<float> tf((size_t)NCLS * 16);
    std::vector<uint32_t> tq((size_t)NCLS * 16 * 2);
    for (int cls = 0; cls < NCLS; ++cls)
        for (int j = 0; j < 16; ++j) {
            const int dy = j < 15 ? abs(j - 7) : 7;
            const float a = T[cls * GY + dy];
            tf[cls * 16 + j] = a;
            const uint16_t h1 = bf16_rne(a);
            const float r1 = a - bf2f(h1);
            const uint16_t h2 = bf16_rne(r1);
            const uint16_t h3 = bf16_rne(r1 - bf2f(h2));
            tq[(cls * 16 + j) * 2] = (uint32_t)h1 | ((uint32_t)h2 << 16);
            tq[(cls * 16 + j) * 2 + 1] = h3;
        }
    float *dA, *dO, *dTf;
    uint16_t* dS;
    uint32_t* dTq;
    const size_t outn = (size_t)nwg * NT * TPW * 16;
    hipMalloc(&dA, hA.size() * 4);
    hipMalloc(&dS, hS.size() * 2);
    hipMalloc(&dTf, tf.size() * 4);
    hipMalloc(&dTq, tq.size() * 4);
    hipMalloc(&dO, outn * 4);
    hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dS, hS.data(), hS.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dTf, tf.data(), tf.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dTq, tq.data(), tq.size() * 4, hipMemcpyHostToDevice);
    const char* names[5] = {"f32_stream", "f32_table", "split_stream", "split_table", "split_noload"};
    std::vector<std::vector<float>> res(5, std::vector<float>(outn));
    double tf_[5];
    tf_[0] = run<0>(dA, dS, dTf, dO, nwg, reps);
    hipMemcpy(res[0].data(), dO, outn * 4, hipMemcpyDeviceToHost);
    tf_[1] = run<1>(dA, dS, dTf, dO, nwg, reps);
    hipMemcpy(res[1].data(), dO, outn * 4, hipMemcpyDeviceToHost);
    tf_[2] = run<2>(dA, dS, dTq, dO, nwg, reps);
    hipMemcpy(res[2].data(), dO, outn * 4, hipMemcpyDeviceToHost);
    tf_[3] = run<3>(dA, dS, dTq, dO, nwg, reps);
    hipMemcpy(res[3].data(), dO, outn * 4, hipMemcpyDeviceToHost);
    tf_[4] = run<4>(dA, dS, dTq, dO, nwg, reps);
    for (int v = 0; v < 5; ++v) printf("%-13s %7.2f TFLOP/s (fp32-equivalent; fp32 MFMA peak 157.3)\n", names[v], tf_[v]);
    long d01 = 0, d23 = 0;
    for (size_t i = 0; i < outn; ++i) {
        d01 += memcmp(&res[0][i], &res[1][i], 4) != 0;
        d23 += memcmp(&res[2][i], &res[3][i], 4) != 0;
    }
    printf("bitwise mismatches: f32_table vs f32_stream %ld, split_table vs split_stream %ld (of %zu)\n", d01, d23,
           outn);
    // accuracy vs the exact sum on workgroups 0 and 255 (every output)
    double e0 = 0, e2 = 0, s0 = 0, s2 = 0;
    long cnt = 0;
    for (int w : {0, 255})
        for (int tid = 0; tid < NT; ++tid)
            for (int t = 0; t < TPW; ++t)
                for (int r = 0; r < 16; ++r) {
                    const int l = tid & 63, wave = tid >> 6;
                    const int row = (r % 4) + 8 * (r / 4) + 4 * (l >> 5), col = (wave * TPW + t) * 32 + (l & 31);
                    long double ex = 0;
                    for (int k = 0; k < N; ++k) ex += (long double)h_operand(row, k, w) * alpha[(size_t)k * N + col];
                    const size_t o = ((size_t)(w * NT + tid) * TPW + t) * 16 + r;
                    const double a0 = fabs((double)(res[0][o] - ex)), a2 = fabs((double)(res[2][o] - ex));
                    e0 = a0 > e0 ? a0 : e0;
                    e2 = a2 > e2 ? a2 : e2;
                    s0 += a0;
                    s2 += a2;
                    ++cnt;
                }
    if (argc > 2) {
        FILE* f = fopen(argv[2], "wb");
        if (!f) return 1;
        fwrite(res[2].data(), 4, (size_t)NT * TPW * 16, f);
        fclose(f);
    }
    if (argc > 3) {
        float* dTr;
        const size_t trn = (size_t)NKB * 6 * 64 * 16;
        hipMalloc(&dTr, trn * 4);
        hipLaunchKernelGGL(trace, dim3(1), dim3(64), 0, 0, dS, dTr);
        std::vector<float> htr(trn);
        hipMemcpy(htr.data(), dTr, trn * 4, hipMemcpyDeviceToHost);
        FILE* f = fopen(argv[3], "wb");
        if (!f) return 1;
        fwrite(htr.data(), 4, trn, f);
        fclose(f);
    }
    printf("|error| vs exact over %ld outputs: f32 max %.3g mean %.3g; split max %.3g mean %.3g\n", cnt, e0, s0 / cnt,
           e2, s2 / cnt);
    return 0;
}
