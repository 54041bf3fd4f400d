// kura_detmath.h -- deterministic IEEE-754 primitives for the Kuramoto step.
//
// Why this file exists: the reference RHS (environment/env.py:252-256) is
// integrated by an adaptive Dopri5 whose dense-output polynomial cancels
// catastrophically in fp32 (diffrax FourthOrderPolynomialInterpolation, see
// DESIGN.md "Numerics"). A 1-ulp difference anywhere in the pipeline grows
// to ~1 rad after 1000 env-steps, so the 1e-5-relative phase gate of
// BASELINE.json can only be met by a GPU path that is a *bit-exact twin* of
// the CPU oracle. Every transcendental used on the path is therefore defined
// here from +,-,*,fma,rint,trunc only (all exactly specified by IEEE-754 on
// both gfx950 and x86-64), and the same header is compiled by hipcc (device)
// and gcc (oracle/). Both sides must be built with -ffp-contract=off.
//
// Accuracy (checked by tests/test_detmath.py against libm in double):
//   kdm_sincosf  <= 2 ulp on |x| < 1e4 (Cody-Waite 3-part pi/2, Cephes polys)
//   kdm_fmod2pi  exact (== fmodf(y, (float)(2*pi)), as jnp.fmod in env.py:253)
//   kdm_inv_fifth_root  ~0.5 ulp after rounding to float
#pragma once

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define KDM_FN __host__ __device__ static inline
#define KDM_FMAF(a, b, c) __builtin_fmaf((a), (b), (c))
#define KDM_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#include <math.h>
#include <stdint.h>
#define KDM_FN static inline
#define KDM_FMAF(a, b, c) fmaf((a), (b), (c))
#define KDM_FMA(a, b, c) fma((a), (b), (c))
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

// (float)(2*pi): jnp.fmod(y, 2*jnp.pi) with x64 disabled divides by this.
#define KDM_TWO_PI_F 6.28318548202514648438f      /* 0x1.921fb6p+2 */
#define KDM_INV_TWO_PI_F 0.15915493667125701904f  /* 0x1.45f306p-3 */
#define KDM_TWO_OVER_PI_F 0.63661974668502807617f /* 0x1.45f306p-1 */
// pi/2 = C1 + C2 + C3 (+1e-23), each a float; products with an integer
// quadrant count are exact inside fmaf.
#define KDM_PIO2_C1 1.57079637050628662109f       /* 0x1.921fb6p+0 */
#define KDM_PIO2_C2 (-4.37113882867379290890e-08f) /* -0x1.777a5cp-25 */
#define KDM_PIO2_C3 (-1.71512451884415714046e-15f) /* -0x1.ee59dap-50 */

// Exact fmodf(y, KDM_TWO_PI_F).  Result has the sign of y (C / jnp.fmod).
// For |y| < 2^22 the quotient estimate is off by at most one and the
// remainder computed by fmaf is exact; larger |y| takes the
// classic shift-subtract path, which is exact by Sterbenz's lemma.
// Fast path of kdm_fmod2pi, exact for |y| < 2^22 (sets *slow otherwise; the
// caller then re-evaluates that element with kdm_fmod2pi).  Branch-free, so a
// batch of elements keeps its instruction-level parallelism.
KDM_FN float kdm_fmod2pi_fast(float y, int* slow) {
    const float d = KDM_TWO_PI_F;
    const float ay = fabsf(y);
    const float q = truncf(ay * KDM_INV_TWO_PI_F);
    float r = KDM_FMAF(-q, d, ay);
    r = r < 0.0f ? r + d : r;
    r = r >= d ? r - d : r;
    *slow |= !(ay < 4194304.0f);
    return y < 0.0f ? -r : r;
}

KDM_FN float kdm_fmod2pi(float y) {
    int slow = 0;
    const float rf = kdm_fmod2pi_fast(y, &slow);
    if (!slow) return rf;
    // rare (|y| >= 2^22, inf, nan): shift-subtract long division, exact by
    // Sterbenz's lemma
    const float d = KDM_TWO_PI_F;
    float r = fabsf(y);
    if (!(r < 3.0e38f)) return (y - y) / (y - y);  // inf/nan -> nan
    float dd = d;
    int e = 0;
    while (dd * 2.0f <= r) { dd *= 2.0f; ++e; }
    for (; e >= 0; --e) {
        if (r >= dd) r -= dd;
        dd *= 0.5f;
    }
    return y < 0.0f ? -r : r;
}

// sin and cos of x (any float with |x| < ~1e5 for full accuracy).
KDM_FN void kdm_sincosf(float x, float* s_out, float* c_out) {
    float j = rintf(x * KDM_TWO_OVER_PI_F);
    float r = KDM_FMAF(-j, KDM_PIO2_C1, x);
    r = KDM_FMAF(-j, KDM_PIO2_C2, r);
    r = KDM_FMAF(-j, KDM_PIO2_C3, r);
    int q = ((int)j) & 3;
    float z = r * r;
    // Cephes sinf/cosf minimax polynomials on [-pi/4, pi/4]
    float ps = KDM_FMAF(z, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = KDM_FMAF(z, ps, -1.6666654611e-1f);
    float sr = KDM_FMAF(r * z, ps, r);
    float pc = KDM_FMAF(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = KDM_FMAF(z, pc, 4.166664568298827e-2f);
    float cr = KDM_FMAF(z * z, pc, KDM_FMAF(-0.5f, z, 1.0f));
    // quadrant selection without branches (v_cndmask on the GPU):
    // q=0: (s,c) = (sr,cr); 1: (cr,-sr); 2: (-sr,-cr); 3: (-cr,sr)
#ifdef KURA_BITSEL
    // variant (r02 bit-select probe): select on bit patterns + sign-bit xor
    const uint32_t usr = __builtin_bit_cast(uint32_t, sr), ucr = __builtin_bit_cast(uint32_t, cr);
    const uint32_t odd = (uint32_t)(q & 1);
    uint32_t us = odd ? ucr : usr;
    uint32_t uc = odd ? usr : ucr;
    us ^= ((uint32_t)q & 2u) << 30;
    uc ^= ((uint32_t)(q + 1) & 2u) << 30;
    float s = __builtin_bit_cast(float, us);
    float c = __builtin_bit_cast(float, uc);
#else
    float s = (q & 1) ? cr : sr;
    float c = (q & 1) ? sr : cr;
    s = (q & 2) ? -s : s;
    c = ((q + 1) & 2) ? -c : c;
#endif
    *s_out = s;
    *c_out = c;
}


// sin and cos of fmod(y, 2pi_f) -- env.py:253-255's theta = jnp.fmod(y, 2*pi)
// followed by the sin of phase differences (factorised into sin/cos of theta)
// -- with the 2pi_f reduction folded into the Cody-Waite reduction.
// 2pi_f = (float)(2 pi) = 4 * C1 exactly.  With k = trunc(y / 2pi_f) (fmod's
// quotient, estimated as trunc(y * (1/2pi)_f) without fmod's exact
// correction steps), n = rint(y * 2/pi_f) and j = n - 4k:
//     r = y - n*C1 - j*C2 - j*C3 = (y - k*2pi_f) - j*(C1 + C2 + C3),
// the Cody-Waite remainder of theta_k = y - k*2pi_f with quadrant j & 3.
// That is fmod(y, 2pi_f)'s remainder whenever the estimated k is fmod's
// quotient; it is off by one only for y within a few ulp(y) of a multiple of
// 2pi_f (theta within ~1e-3 rad of 0 or 2pi_f at |y| ~ 5e3), where the sine's
// argument then moves by 2pi - 2pi_f = 1.7e-7 rad -- inside the RHS pin
// against the reference's op sequence (tests/test_golden_reference.py).
// fmaf(-n, C1, y) is exact-then-rounded-once, like fmaf(-j, C1, fmod(y)) in
// the unfolded form, so away from those points the result is the unfolded
// one's accuracy; the separate fmod pass and its corrections are gone (the
// stage input's VALU work per element drops by about a sixth).  Valid for
// |y| < 2^22; the piecewise definition below takes the exact fmod +
// kdm_sincosf path beyond (never reached in practice: ~4e6 rad).
KDM_FN void kdm_sincos_red(float r, int q, float* s_out, float* c_out) {
    float z = r * r;
    float ps = KDM_FMAF(z, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = KDM_FMAF(z, ps, -1.6666654611e-1f);
    float sr = KDM_FMAF(r * z, ps, r);
    float pc = KDM_FMAF(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = KDM_FMAF(z, pc, 4.166664568298827e-2f);
    float cr = KDM_FMAF(z * z, pc, KDM_FMAF(-0.5f, z, 1.0f));
    float s = (q & 1) ? cr : sr;
    float c = (q & 1) ? sr : cr;
    s = (q & 2) ? -s : s;
    c = ((q + 1) & 2) ? -c : c;
    *s_out = s;
    *c_out = c;
}

// fast path (|y| < 2^22; sets *slow otherwise): reduced argument and quadrant
KDM_FN float kdm_fold_reduce(float y, int* q, int* slow) {
    const float k = truncf(y * KDM_INV_TWO_PI_F);
    const float n = rintf(y * KDM_TWO_OVER_PI_F);
    const int j = (int)n - 4 * (int)k;
    const float jf = (float)j;
    float r = KDM_FMAF(-n, KDM_PIO2_C1, y);
    r = KDM_FMAF(-jf, KDM_PIO2_C2, r);
    r = KDM_FMAF(-jf, KDM_PIO2_C3, r);
    *q = j & 3;
    *slow |= !(fabsf(y) < 4194304.0f);
    return r;
}

KDM_FN void kdm_sincos_fmod2pi(float y, float* s_out, float* c_out) {
    int slow = 0, q;
    const float r = kdm_fold_reduce(y, &q, &slow);
    if (!slow) {
        kdm_sincos_red(r, q, s_out, c_out);
        return;
    }
    kdm_sincosf(kdm_fmod2pi(y), s_out, c_out);  // |y| >= 2^22, inf, nan
}

KDM_FN float kdm_cosf(float x) {
    float s, c;
    kdm_sincosf(x, &s, &c);
    return c;
}

// x^(-1/5) for finite x > 0, rounded to float.  Only +,*,fma and exact
// power-of-two scaling are used, so host and device agree bit for bit.
// Special values follow pow(): x == 0 -> +inf, x == +inf -> 0, nan -> nan.
KDM_FN float kdm_inv_fifth_root(float xf) {
    if (xf != xf) return xf;
    if (xf <= 0.0f) return (xf == 0.0f) ? __builtin_inff() : (xf - xf) / (xf - xf);
    if (xf > 3.40282346638528859812e+38f) return 0.0f;
    // decompose x = m * 2^e with m in [1, 2) using the float bit pattern
    union { float f; uint32_t u; } cv;
    cv.f = xf;
    int e;
    double m;
    uint32_t bexp = (cv.u >> 23) & 0xffu;
    if (bexp == 0) {  // subnormal float: normalise in double
        double xd = (double)xf * 18014398509481984.0;  // 2^54
        union { double d; uint64_t u; } dv;
        dv.d = xd;
        e = (int)((dv.u >> 52) & 0x7ffu) - 1023 - 54;
        dv.u = (dv.u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;
        m = dv.d;
    } else {
        e = (int)bexp - 127;
        union { float f; uint32_t u; } mv;
        mv.u = (cv.u & 0x007fffffu) | 0x3f800000u;
        m = (double)mv.f;
    }
    // e = 5*q + r with r in [0, 5)
    int qd = (e >= 0) ? e / 5 : -((-e + 4) / 5);
    int r = e - 5 * qd;
    // w ~ m^(-1/5) on [1, 2): linear start (rel err < 1.2%) + Newton
    //   w <- w * (1 + (1 - m w^5) / 5)
    double w = KDM_FMA(-0.1236, m, 1.1195);
    for (int it = 0; it < 6; ++it) {
        double w2 = w * w;
        double w5 = w2 * w2 * w;
        double t = KDM_FMA(-m, w5, 1.0);
        w = KDM_FMA(w * 0.2, t, w);
    }
    // 2^(-r/5) for r = 0..4 (a select chain, not an indexed table: on the GPU a
    // run-time-indexed local array lives in scratch memory)
    const double inv_r = r == 0 ? 1.0
                         : r == 1 ? 0x1.bdb8cdadbe120p-1
                         : r == 2 ? 0x1.8406003b2ae5cp-1
                         : r == 3 ? 0x1.51cb453b9536cp-1
                                  : 0x1.2611186bae675p-1;
    double y = w * inv_r;
    // multiply by 2^(-qd) exactly (|qd| <= 30 for float inputs)
    union { double d; uint64_t u; } sc;
    sc.u = (uint64_t)(1023 - qd) << 52;
    return (float)(y * sc.d);
}

// ---- canonical reductions ---------------------------------------------
// Two summation orders are part of the numerics contract (the oracle replays
// both sequentially, oracle/kura_oracle.c):
// RM  (sums over the N oscillators inside the solver: error norm, LFP) --
//     the MFMA accumulator layout of the kernel: wave w (0..7) owns columns
//     32*(w*TPW + t) + c, TPW = N/256; each column lane c sums its TPW values
//     in t order from +0, the 32 lanes combine by an xor butterfly
//     (16,8,4,2,1: p[c] = p[c] + p[c^o]), then the 8 wave totals are added in
//     wave order from +0.  N > 1024: each part of 1024 oscillators (one
//     workgroup of a split group) reduces that way and the part totals are
//     added in part order from +0.
// R64 (sums over the W-sample window: DFT bins, filtfilt mean) -- lane l
//     (0..63) sums x[l], x[l+64], ... from +0, then an xor butterfly with
//     offsets 32,16,8,4,2,1.
