// kura_r2.h -- the R2 reward's filter term as a linear functional of the window.
//
// reward_temp_const_lfp_betafilt_action (environment/env.py:653-666) takes
//     f = band_pass_envelope(x)  ->  scipy.signal.filtfilt(b, a, x)
// (environment/utils.py:794-816: butter(2, [12, 30]/(fs/2), 'band'), padtype
// 'odd', padlen = 3*max(len(a), len(b)) = 15, each lfilter pass started from
// lfilter_zi(b, a) * (its first input)) and uses only
//     d = f[-1] - mean(f),     R2 = -1e3 * d^2 - 1e-2 * |u|.
// Every stage of that -- odd extension, both DF2T passes with their
// input-scaled initial states, the reversal, the crop, last-minus-mean -- is
// linear in the window x, so d = c . x for one vector c in R^W that depends
// only on (b, a, zi, W, padlen).  kura_r2_functional computes c in O(W) by
// running the adjoint of that chain on the functional g = e_last - 1/W:
//     pass:   v = T u + r u[0]     (T: the filter's lower-triangular impulse
//                                   response, r: its zero-input response from
//                                   the state zi)
//     adjoint: gu = T^T g + e_0 (r . g),   T^T g = rev(lfilter(b, a, rev(g)))
// followed by the transpose of the odd extension.  The step kernel then needs
// one W-long dot product per env (the shape of one DFT bin) instead of two
// serial 2370-sample IIR recursions.
//
// c is accumulated in long double (x87 80-bit on x86-64, the same on gcc and
// clang: +, -, * only) and rounded to float64 once: the adjoint filters'
// poles sit close to the unit circle, and in float64 c . x came out ~6x less
// accurate than scipy's own filtfilt (3e-11 vs 4e-12 relative against an
// extended-precision filtfilt); with the extended accumulation it is ~1e-15.
//
// Shared by the host side of libkura (kura_capi.inc) and the CPU oracle
// (oracle/kura_oracle.c): both build c with this code, so the GPU and the
// oracle take the same dot product with the same c, bit for bit.  c agrees
// with the filtfilt it replaces to float64 rounding (tests/test_r2_functional.py,
// and the reference's own scipy values in tests/golden).  Plain C, no
// contraction (-ffp-contract=off on both compilers).
#pragma once

#include <stdlib.h>
#include <string.h>

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

typedef long double kura_r2_real;

// y = lfilter(b, a, x) (scipy DF2T, 5 taps, a[0] == 1) started from state z
// (z is advanced in place).
static inline void kura_r2_lfilter(const kura_r2_real* b, const kura_r2_real* a, const kura_r2_real* x,
                                   kura_r2_real* y, int n, kura_r2_real* z) {
    for (int k = 0; k < n; ++k) {
        const kura_r2_real xn = x[k];
        const kura_r2_real yn = z[0] + b[0] * xn;
        z[0] = (z[1] + xn * b[1]) - yn * a[1];
        z[1] = (z[2] + xn * b[2]) - yn * a[2];
        z[2] = (z[3] + xn * b[3]) - yn * a[3];
        z[3] = xn * b[4] - yn * a[4];
        y[k] = yn;
    }
}

// g (length L) <- the adjoint of one filtfilt pass applied to g: T^T g +
// e_0 (r . g).  t, s: L doubles of scratch.
static inline void kura_r2_pass_adjoint(const kura_r2_real* b, const kura_r2_real* a, const kura_r2_real* zi,
                                        kura_r2_real* g, int L, kura_r2_real* t, kura_r2_real* s) {
    // r . g, r = zero-input response from the state zi
    kura_r2_real z[4] = {zi[0], zi[1], zi[2], zi[3]};
    for (int k = 0; k < L; ++k) t[k] = 0.0;
    kura_r2_lfilter(b, a, t, s, L, z);
    kura_r2_real rg = 0.0L;
    for (int k = 0; k < L; ++k) rg = rg + s[k] * g[k];
    // T^T g = rev(lfilter(rev(g)))
    for (int k = 0; k < L; ++k) t[k] = g[L - 1 - k];
    kura_r2_real z0[4] = {0.0L, 0.0L, 0.0L, 0.0L};
    kura_r2_lfilter(b, a, t, s, L, z0);
    for (int k = 0; k < L; ++k) g[k] = s[L - 1 - k];
    g[0] = g[0] + rg;
}

// c[0..W) with filtfilt(b, a, x)[-1] - mean(filtfilt(b, a, x)) == c . x
// (padtype 'odd', padlen P, 0 < P < W).  Returns 0, or -1 on bad sizes /
// allocation failure.
static inline int kura_r2_functional(const double* b, const double* a, const double* zi, int W, int P, double* c) {
    if (W < 2 || P < 1 || P >= W) return -1;
    const int L = W + 2 * P;
    kura_r2_real* g = (kura_r2_real*)malloc(sizeof(kura_r2_real) * ((size_t)L * 3 + W));
    if (!g) return -1;
    kura_r2_real* t = g + L;
    kura_r2_real* s = t + L;
    kura_r2_real* cl = s + L;
    kura_r2_real bl[5], al[5], zl[4];
    for (int i = 0; i < 5; ++i) {
        bl[i] = b[i];
        al[i] = a[i];
    }
    for (int i = 0; i < 4; ++i) zl[i] = zi[i];
    // functional on the second pass's output v: f[i] = v[L-1-P-i], i < W;
    // d = f[W-1] - (1/W) sum_i f[i] = v[P] - (1/W) sum_{m=P}^{P+W-1} v[m]
    for (int m = 0; m < L; ++m) g[m] = 0.0;
    const kura_r2_real inv = 1.0L / (kura_r2_real)W;
    for (int m = P; m < P + W; ++m) g[m] = -inv;
    g[P] = g[P] + 1.0L;
    // second pass (input u = rev(y)), the reversal, the first pass (input ext)
    kura_r2_pass_adjoint(bl, al, zl, g, L, t, s);
    for (int k = 0; k < L; ++k) t[k] = g[L - 1 - k];
    memcpy(g, t, sizeof(kura_r2_real) * (size_t)L);
    kura_r2_pass_adjoint(bl, al, zl, g, L, t, s);
    // odd extension: ext[k] = 2 x[0] - x[P-k] (k < P), x[k-P] (P <= k < P+W),
    // 2 x[W-1] - x[W-2-(k-P-W)] (k >= P+W)
    for (int i = 0; i < W; ++i) cl[i] = g[P + i];
    for (int k = 0; k < P; ++k) {
        cl[0] = cl[0] + 2.0L * g[k];
        cl[P - k] = cl[P - k] - g[k];
    }
    for (int k = P + W; k < L; ++k) {
        cl[W - 1] = cl[W - 1] + 2.0L * g[k];
        cl[W - 2 - (k - P - W)] = cl[W - 2 - (k - P - W)] - g[k];
    }
    for (int i = 0; i < W; ++i) c[i] = (double)cl[i];
    free(g);
    return 0;
}
