// Probe of v_mfma_f32_32x32x16_bf16's accumulation semantics on gfx950
// (groundwork for a split-bf16 coupling GEMM): how the
// 16 exact bf16 x bf16 products of one output and the f32 accumulator input
// are summed and rounded.  Output D[0][0] of one MFMA with A row 0 = x (16
// values), B column 0 = y, C[0][0] = c, for many random trials; the host
// compares it with candidate models:
//   exact  : round_f32(c + sum of the exact products)            (one rounding)
//   seq_k  : fmaf chain from c over k = 0..15                     (16 roundings)
//   seq_rk : fmaf chain from c over k = 15..0
//   sum_c  : round_f32(round_f32(sum of products) + c)
// Lane mapping assumed: A[l%32][8*(l/32) + i], B[8*(l/32) + i][l%32] for the
// 8 bf16 of lane l; D value j of lane l at row (j%4) + 8*(j/4) + 4*(l/32),
// column l%32.  (Only the seq_* models depend on the k order.)
//   hipcc --offload-arch=gfx950 -O2 -o tools/mfma_bf16_probe tools/mfma_bf16_probe.hip
//   ./mfma_bf16_probe [trials] [dump.bin] [f16]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const uint16_t* x, const uint16_t* y, const float* c, float* out, int trials, int f16) {
    const int l = threadIdx.x;
    for (int t = 0; t < trials; ++t) {
        bf16x8 a, b;
        f16x8 ah, bh;
        for (int i = 0; i < 8; ++i) {
            const int k = 8 * (l / 32) + i;
            const uint16_t xa = (l % 32 == 0) ? x[t * 16 + k] : 0;
            const uint16_t yb = (l % 32 == 0) ? y[t * 16 + k] : 0;
            a[i] = __builtin_bit_cast(__bf16, xa);
            b[i] = __builtin_bit_cast(__bf16, yb);
            ah[i] = __builtin_bit_cast(_Float16, xa);
            bh[i] = __builtin_bit_cast(_Float16, yb);
        }
        f32x16 acc;
        for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
        if (l == 0) acc[0] = c[t];
        if (f16) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
        else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        if (l == 0) out[t] = acc[0];
    }
}

static float h2f(uint16_t h) {   // IEEE binary16 -> float (normal and subnormal)
    const int s = h >> 15, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    float v = e == 0 ? ldexpf((float)m, -24) : ldexpf((float)(m | 0x400), e - 25);
    return s ? -v : v;
}

static uint16_t rnd_f16(unsigned* s, int emin, int emax) {
    *s = *s * 1664525u + 1013904223u;
    const unsigned r = *s >> 8;
    const int e = emin + (int)(r % (unsigned)(emax - emin + 1));
    const unsigned m = (r >> 6) & 0x3ff;
    const unsigned sg = (r >> 16) & 1;
    return (uint16_t)((sg << 15) | ((unsigned)(e + 15) << 10) | m);
}

static float bf2f(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static uint16_t rnd_bf16(unsigned* s, int emin, int emax) {
    *s = *s * 1664525u + 1013904223u;
    const unsigned r = *s >> 8;
    const int e = emin + (int)(r % (unsigned)(emax - emin + 1));
    const unsigned m = (r >> 8) & 0x7f;
    const unsigned sg = (r >> 15) & 1;
    return (uint16_t)((sg << 15) | ((unsigned)(e + 127) << 7) | m);
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 20000;
    const int f16 = argc > 3 && strcmp(argv[3], "f16") == 0;   // v_mfma_f32_32x32x16_f16 instead
    uint16_t *hx = (uint16_t*)malloc(trials * 16 * 2), *hy = (uint16_t*)malloc(trials * 16 * 2);
    float *hc = (float*)malloc(trials * 4), *ho = (float*)malloc(trials * 4);
    unsigned s = 12345;
    for (int t = 0; t < trials; ++t) {
        // mixed regimes: wide exponent spread (cancellation / absorption), narrow spread
        const int wide = t % 3;
        for (int k = 0; k < 16; ++k) {
            if (f16) {
                hx[t * 16 + k] = wide ? rnd_f16(&s, -12, 6) : rnd_f16(&s, -2, 2);
                hy[t * 16 + k] = wide == 2 ? rnd_f16(&s, -12, 6) : rnd_f16(&s, -1, 1);
            } else {
                hx[t * 16 + k] = wide ? rnd_bf16(&s, -12, 6) : rnd_bf16(&s, -2, 2);
                hy[t * 16 + k] = wide == 2 ? rnd_bf16(&s, -12, 6) : rnd_bf16(&s, -1, 1);
            }
        }
        const uint16_t cb = rnd_bf16(&s, -8, 8);
        hc[t] = (t % 4 == 0) ? 0.0f : bf2f(cb) * 1.0000001f;
    }
    uint16_t *dx, *dy;
    float *dc, *dout;
    hipMalloc(&dx, trials * 32);
    hipMalloc(&dy, trials * 32);
    hipMalloc(&dc, trials * 4);
    hipMalloc(&dout, trials * 4);
    hipMemcpy(dx, hx, trials * 32, hipMemcpyHostToDevice);
    hipMemcpy(dy, hy, trials * 32, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc, trials * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dx, dy, dc, dout, trials, f16);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    hipMemcpy(ho, dout, trials * 4, hipMemcpyDeviceToHost);
    long m_exact = 0, m_seqk = 0, m_seqr = 0, m_sumc = 0, m_any = 0;
    int shown = 0;
    for (int t = 0; t < trials; ++t) {
        long double ex = hc[t];
        long double ps = 0.0L;
        float fk = hc[t], fr = hc[t];
        for (int k = 0; k < 16; ++k) {
            const float xv = f16 ? h2f(hx[t * 16 + k]) : bf2f(hx[t * 16 + k]);
            const float yv = f16 ? h2f(hy[t * 16 + k]) : bf2f(hy[t * 16 + k]);
            const float p = xv * yv;   // exact in f32 (8x8- or 11x11-bit mantissas)
            ex += (long double)p;
            ps += (long double)p;
            fk = fmaf(xv, yv, fk);
        }
        for (int k = 15; k >= 0; --k) {
            const float xv = f16 ? h2f(hx[t * 16 + k]) : bf2f(hx[t * 16 + k]);
            const float yv = f16 ? h2f(hy[t * 16 + k]) : bf2f(hy[t * 16 + k]);
            fr = fmaf(xv, yv, fr);
        }
        const float e1 = (float)ex, e4 = (float)((float)ps + hc[t]);
        const float g = ho[t];
        const int a = g == e1, b = g == fk, c2 = g == fr, d = g == e4;
        m_exact += a;
        m_seqk += b;
        m_seqr += c2;
        m_sumc += d;
        m_any += a | b | c2 | d;
        if (!(a | b | c2 | d) && shown < 8) {
            printf("trial %d: gpu %.9g exact %.9g seq_k %.9g seq_rk %.9g sum_c %.9g\n", t, g, e1, fk, fr, e4);
            ++shown;
        }
    }
    printf("trials %d: exact %ld  seq_k %ld  seq_rk %ld  sum_c %ld  any %ld\n", trials, m_exact, m_seqk, m_seqr,
           m_sumc, m_any);
    if (argc > 2) {   // raw dump for offline model fitting: x, y (uint16 x 16 per trial), c, gpu (f32 per trial)
        FILE* f = fopen(argv[2], "wb");
        if (!f) return 1;
        fwrite(hx, 2, (size_t)trials * 16, f);
        fwrite(hy, 2, (size_t)trials * 16, f);
        fwrite(hc, 4, (size_t)trials, f);
        fwrite(ho, 4, (size_t)trials, f);
        fclose(f);
    }
    return 0;
}
