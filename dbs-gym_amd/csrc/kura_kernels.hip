// kura_kernels.hip -- fused CDNA4 (gfx950) kernels for the batched Kuramoto
// environment: one launch = one SpatialKuramoto.step() (env.py:415-454) or
// one reset() transient (env.py:594-614) for every environment of a handle.
//
// Work decomposition (DESIGN.md "Kernel K1"):
//   * one workgroup = 16 environments (E_WG), 512 threads = 8 wavefronts;
//   * the O(N^2) coupling of one RHS sweep is the GEMM
//         [sin theta ; cos theta] (32 x N)  x  alpha^T (N x N)
//     on v_mfma_f32_32x32x2_f32 (exact fp32, k-ordered fmaf chain), with the
//     32 x N operand resident in LDS (128 KiB at N=1024) in MFMA fragment order
//     and alpha streamed from L2/MALL in a host-swizzled fragment layout;
//   * every element-wise / reduction stage (Dopri5 stage inputs, error norm,
//     dense output, LFP, window, reward) runs in the "R64" layout: wave w owns
//     envs {2w, 2w+1}, lane l owns oscillators l, l+64, ...  so each per-env
//     sum is a strided lane loop + xor butterfly (kura_detmath.h), identical
//     to the CPU oracle's order.
// The arithmetic is a bit-exact twin of oracle/kura_oracle.c; this file must
// be compiled with -ffp-contract=off (see __graft_entry__.build).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kura.h"
#include "kura_detmath.h"

#pragma clang fp contract(off)

#define E_WG 16
#define NWAVES 8
#define NTHREADS (NWAVES * 64)
#define ENVS_PER_WAVE (E_WG / NWAVES)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---- Dopri5 tableau cast to fp32 (identical constants to the oracle) -------
#define KF(x) ((float)(x))
__constant__ static const float kA21 = KF(1.0 / 5.0);
__constant__ static const float kA31 = KF(3.0 / 40.0), kA32 = KF(9.0 / 40.0);
__constant__ static const float kA41 = KF(44.0 / 45.0), kA42 = KF(-56.0 / 15.0), kA43 = KF(32.0 / 9.0);
__constant__ static const float kA51 = KF(19372.0 / 6561.0), kA52 = KF(-25360.0 / 2187.0),
                                kA53 = KF(64448.0 / 6561.0), kA54 = KF(-212.0 / 729.0);
__constant__ static const float kA61 = KF(9017.0 / 3168.0), kA62 = KF(-355.0 / 33.0),
                                kA63 = KF(46732.0 / 5247.0), kA64 = KF(49.0 / 176.0),
                                kA65 = KF(-5103.0 / 18656.0);
__constant__ static const float kA71 = KF(35.0 / 384.0), kA73 = KF(500.0 / 1113.0), kA74 = KF(125.0 / 192.0),
                                kA75 = KF(-2187.0 / 6784.0), kA76 = KF(11.0 / 84.0);
__constant__ static const float kE1 = KF(35.0 / 384.0 - 1951.0 / 21600.0),
                                kE3 = KF(500.0 / 1113.0 - 22642.0 / 50085.0),
                                kE4 = KF(125.0 / 192.0 - 451.0 / 720.0),
                                kE5 = KF(-2187.0 / 6784.0 + 12231.0 / 42400.0),
                                kE6 = KF(11.0 / 84.0 - 649.0 / 6300.0), kE7 = KF(-1.0 / 60.0);
__constant__ static const float kM1 = KF(6025192743.0 / 30085553152.0 / 2.0),
                                kM3 = KF(51252292925.0 / 65400821598.0 / 2.0),
                                kM4 = KF(-2691868925.0 / 45128329728.0 / 2.0),
                                kM5 = KF(187940372067.0 / 1594534317056.0 / 2.0),
                                kM6 = KF(-1776094331.0 / 19743644256.0 / 2.0),
                                kM7 = KF(11237099.0 / 235043384.0 / 2.0);
#undef KF

// Everything a launch needs, passed by value (kernarg).
struct DevParams {
    int N, B, W, n_elec, n_rec, rec_kernel, reward_kind, episode_steps, max_steps, n_bins, padlen;
    int bins[KURA_MAX_BINS];
    double dt, width, pause, transient_len, act_lo, act_hi, dbs_lo, dbs_hi;
    double bw_b[5], bw_a[5], bw_zi[4];
    float rtol, atol, kn, dt0;
    const float* alpha_sw;  // B-fragment swizzled coupling
    const float* omega;     // [B][N]
    const double* g_stim;   // [B][n_elec][N]
    const double* g_rec;    // [B][n_rec][N]
    const double* ctab;     // [n_bins][W]
    const double* stab;
    float* y;               // [B][N] phase state (last saved row)
    double* t;              // [B] current_time
    int* step;              // [B]
    double* ring;           // [B][W] observation window ring
    int* wpos;              // [B] next write slot == oldest sample
    float* F;               // [B][7][N] stage derivatives
    float* Y0;              // [B][N]
    float* Y1;              // [B][N]
    float* pulse;           // [B][N]
    double* scratch;        // [B][W + 2*padlen] * 2 (R2 filtfilt)
    unsigned long long* stats;  // [4]: max rhs, steps, rejected, flags
};

// LDS index of X[row][k] in MFMA A-fragment order: for k-block kb = k/8 the
// 64 lanes' 4 consecutive k-steps are 16 contiguous bytes (one ds_read_b128).
__device__ __forceinline__ int xs_idx(int row, int k) {
    return (((k >> 3) * 64 + row + 32 * (k & 1)) << 2) + ((k >> 1) & 3);
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = v + __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = v + __shfl_xor(v, o, 64);
    return v;
}

struct Grid {
    double start, delta;
    int n;
};
// np.arange(start, stop, step) in float64 (oracle arange()).
__device__ __forceinline__ Grid make_grid(double start, double stop, double step) {
    Grid g;
    double len = ceil((stop - start) / step);
    g.n = len > 0.0 ? (int)len : 0;
    g.start = start;
    g.delta = (start + step) - start;
    return g;
}
__device__ __forceinline__ double grid_at(const Grid& g, int i) {
    return i == 0 ? g.start : g.start + (double)i * g.delta;
}

// Per-env solver control (wave-uniform; lives in the owning wave).
struct Ctl {
    Grid g;
    float t1, tprev, tnext, h;
    int si, active, nsteps, rejected, flags;
    int lfp_from, lfp_to, pos0;  // which saved rows feed LFP samples, and where
};

// ---------------------------------------------------------------- GEMM ----
// acc[t] (32 x 32 tile, columns jt = wave*TPW + t) = X (LDS) x B-fragments.
template <int TPW>
__device__ __forceinline__ void coupling_gemm(const float* __restrict__ Xs, const float* __restrict__ alpha_sw,
                                              int N, floatx16 (&acc)[TPW]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int NK8 = N >> 3;
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
    const floatx4* xs4 = reinterpret_cast<const floatx4*>(Xs);
    const floatx4* bp[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
        bp[t] = reinterpret_cast<const floatx4*>(alpha_sw) + ((size_t)(wave * TPW + t) * NK8) * 64 + lane;
    floatx4 bcur[TPW], bnxt[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) bcur[t] = bp[t][0];
    for (int kb = 0; kb < NK8; ++kb) {
        if (kb + 1 < NK8) {
#pragma unroll
            for (int t = 0; t < TPW; ++t) bnxt[t] = bp[t][(size_t)(kb + 1) * 64];
        }
        floatx4 a = xs4[kb * 64 + lane];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int t = 0; t < TPW; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], bcur[t][s], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < TPW; ++t) bcur[t] = bnxt[t];
    }
}

// f = fmaf(kn, fmaf(c, P, -(s*Q)), omega) + pulse  ->  F[env][stage][i]
template <int TPW>
__device__ __forceinline__ void coupling_epilogue(const DevParams& p, const float* __restrict__ Xs,
                                                  const floatx16 (&acc)[TPW], int env_base, int stage) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int N = p.N;
    const int h = lane >> 5;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int i = 32 * (wave * TPW + t) + (lane & 31);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = (q & 3) + 8 * (q >> 2) + 4 * h;
            const int env = env_base + e;
            if (env >= p.B) continue;
            const float P = acc[t][q], Q = acc[t][q + 8];
            const float s = Xs[xs_idx(e, i)], c = Xs[xs_idx(16 + e, i)];
            const size_t o = (size_t)env * N + i;
            const float tq = s * Q;
            const float coup = __builtin_fmaf(c, P, -tq);
            const float f = __builtin_fmaf(p.kn, coup, p.omega[o]) + p.pulse[o];
            p.F[((size_t)env * 7 + stage) * N + i] = f;
        }
    }
}

// ------------------------------------------------------------ R64 stages ---
// Stage input ys = y0 + chain(a_s,j * h*F_j), then theta = fmod(ys, 2pi) and
// sin/cos into the LDS operand.  Stage 0 is the solve's initial RHS at y0.
template <int EPL>
__device__ __forceinline__ void stage_input(const DevParams& p, float* Xs, const Ctl (&ctl)[ENVS_PER_WAVE],
                                            int env_base, int s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int N = p.N;
#pragma unroll
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        const int e = wave * ENVS_PER_WAVE + ee;
        const int env = env_base + e;
        if (env >= p.B || !ctl[ee].active) continue;
        const float h = ctl[ee].h;
        const float* Fe = p.F + (size_t)env * 7 * N;
        const float* y0 = p.Y0 + (size_t)env * N;
#pragma unroll 4
        for (int m = 0; m < EPL; ++m) {
            const int i = lane + 64 * m;
            float ys;
            if (s == 0) {
                ys = y0[i];
            } else {
                const float k0 = h * Fe[i];
                float acc;
                switch (s) {
                    case 1: acc = kA21 * k0; break;
                    case 2: acc = kA31 * k0; acc = __builtin_fmaf(kA32, h * Fe[N + i], acc); break;
                    case 3:
                        acc = kA41 * k0;
                        acc = __builtin_fmaf(kA42, h * Fe[N + i], acc);
                        acc = __builtin_fmaf(kA43, h * Fe[2 * N + i], acc);
                        break;
                    case 4:
                        acc = kA51 * k0;
                        acc = __builtin_fmaf(kA52, h * Fe[N + i], acc);
                        acc = __builtin_fmaf(kA53, h * Fe[2 * N + i], acc);
                        acc = __builtin_fmaf(kA54, h * Fe[3 * N + i], acc);
                        break;
                    case 5:
                        acc = kA61 * k0;
                        acc = __builtin_fmaf(kA62, h * Fe[N + i], acc);
                        acc = __builtin_fmaf(kA63, h * Fe[2 * N + i], acc);
                        acc = __builtin_fmaf(kA64, h * Fe[3 * N + i], acc);
                        acc = __builtin_fmaf(kA65, h * Fe[4 * N + i], acc);
                        break;
                    default:
                        acc = kA71 * k0;
                        acc = __builtin_fmaf(kA73, h * Fe[2 * N + i], acc);
                        acc = __builtin_fmaf(kA74, h * Fe[3 * N + i], acc);
                        acc = __builtin_fmaf(kA75, h * Fe[4 * N + i], acc);
                        acc = __builtin_fmaf(kA76, h * Fe[5 * N + i], acc);
                        break;
                }
                ys = y0[i] + acc;
                if (s == 6) p.Y1[(size_t)env * N + i] = ys;
            }
            float sn, cs;
            kdm_sincosf(kdm_fmod2pi(ys), &sn, &cs);
            Xs[xs_idx(e, i)] = sn;
            Xs[xs_idx(16 + e, i)] = cs;
        }
    }
}

// LFP of one saved row (values in registers, R64 layout) -> (naive, records).
template <int EPL>
__device__ __forceinline__ void lfp_of_row(const DevParams& p, int env, const float (&row)[EPL], float* naive,
                                           double* rec) {
    const int lane = threadIdx.x & 63;
    const int N = p.N;
    float cr[EPL];
    float part = 0.0f;
#pragma unroll
    for (int m = 0; m < EPL; ++m) {
        cr[m] = kdm_cosf(row[m]);
        part = part + cr[m];
    }
    const float mean = wave_sum_f32(part) / (float)N;
    *naive = mean;
    if (p.rec_kernel == KURA_REC_GAUSSIAN) {
        double acc = 0.0;
        for (int r = 0; r < p.n_rec; ++r) {
            const double* g = p.g_rec + ((size_t)env * p.n_rec + r) * N;
            double pr = 0.0;
#pragma unroll
            for (int m = 0; m < EPL; ++m) pr = pr + (double)cr[m] * g[lane + 64 * m];
            acc = acc + wave_sum_f64(pr) / (double)N;
        }
        *rec = acc;
    } else {
        *rec = (double)mean;
    }
}

// After the 7th stage: error norm, accept/reject, dense-output saves, FSAL.
// smp_n/smp_r: LDS sample buffers of this env; ring_dst: if non-null, samples
// go straight to the observation ring (reset transient).
template <int EPL>
__device__ __forceinline__ void post_step(const DevParams& p, Ctl& c, int env, float* smp_n, double* smp_r,
                                          double* ring_dst) {
    const int lane = threadIdx.x & 63;
    const int N = p.N;
    const float h = c.h;
    float* Fe = p.F + (size_t)env * 7 * N;
    float* y0p = p.Y0 + (size_t)env * N;
    const float* y1p = p.Y1 + (size_t)env * N;
    // error estimate + RMS norm (R64)
    float part = 0.0f;
#pragma unroll 4
    for (int m = 0; m < EPL; ++m) {
        const int i = lane + 64 * m;
        float e = kE1 * (h * Fe[i]);
        e = __builtin_fmaf(kE3, h * Fe[2 * N + i], e);
        e = __builtin_fmaf(kE4, h * Fe[3 * N + i], e);
        e = __builtin_fmaf(kE5, h * Fe[4 * N + i], e);
        e = __builtin_fmaf(kE6, h * Fe[5 * N + i], e);
        e = __builtin_fmaf(kE7, h * Fe[6 * N + i], e);
        const float a0 = fabsf(y0p[i]), a1 = fabsf(y1p[i]);
        const float mx = a0 > a1 ? a0 : a1;
        const float den = p.atol + mx * p.rtol;
        const float q = e / den;
        part = part + q * q;
    }
    const float mean = wave_sum_f32(part) / (float)N;
    const float err = sqrtf(mean);
    const bool keep = err < 1.0f;
    float fac = 0.9f * kdm_inv_fifth_root(err);
    const float fmn = keep ? 1.0f : 0.2f;
    fac = fac > fmn ? fac : fmn;
    fac = fac < 10.0f ? fac : 10.0f;
    const float dtn = h * fac;
    if (keep) {
        float ca[EPL], cb[EPL], cc[EPL], k0v[EPL], y0v[EPL], y1v[EPL];
#pragma unroll
        for (int m = 0; m < EPL; ++m) {
            const int i = lane + 64 * m;
            const float k0 = h * Fe[i], k6 = h * Fe[6 * N + i];
            float acc = kM1 * k0;
            acc = __builtin_fmaf(kM3, h * Fe[2 * N + i], acc);
            acc = __builtin_fmaf(kM4, h * Fe[3 * N + i], acc);
            acc = __builtin_fmaf(kM5, h * Fe[4 * N + i], acc);
            acc = __builtin_fmaf(kM6, h * Fe[5 * N + i], acc);
            acc = __builtin_fmaf(kM7, k6, acc);
            const float yy0 = y0p[i], yy1 = y1p[i];
            const float ym = yy0 + acc;
            ca[m] = ((2.0f * (k6 - k0)) - (8.0f * (yy1 + yy0))) + (16.0f * ym);
            cb[m] = ((((5.0f * k0) - (3.0f * k6)) + (18.0f * yy0)) + (14.0f * yy1)) - (32.0f * ym);
            cc[m] = (((k6 - (4.0f * k0)) - (11.0f * yy0)) - (5.0f * yy1)) + (16.0f * ym);
            k0v[m] = k0;
            y0v[m] = yy0;
            y1v[m] = yy1;
        }
        while (c.si < c.g.n) {
            const float ts = (float)grid_at(c.g, c.si);
            if (!(ts <= c.tnext)) break;
            const float th = (ts - c.tprev) / (c.tnext - c.tprev);
            float row[EPL];
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                float v = ca[m] * th + cb[m];
                v = v * th + cc[m];
                v = v * th + k0v[m];
                v = v * th + y0v[m];
                row[m] = v;
            }
            if (c.si >= c.lfp_from && c.si < c.lfp_to) {
                float ln;
                double lr;
                lfp_of_row<EPL>(p, env, row, &ln, &lr);
                const int pos = c.si - c.lfp_from + c.pos0;
                if (lane == 0) {
                    if (ring_dst) {
                        ring_dst[pos] = lr;
                    } else {
                        smp_n[pos] = ln;
                        smp_r[pos] = lr;
                    }
                }
            }
            if (c.si == c.g.n - 1) {
#pragma unroll
                for (int m = 0; m < EPL; ++m) p.y[(size_t)env * N + lane + 64 * m] = row[m];
            }
            c.si++;
        }
#pragma unroll
        for (int m = 0; m < EPL; ++m) {
            const int i = lane + 64 * m;
            y0p[i] = y1v[m];
            Fe[i] = Fe[6 * N + i];
        }
        c.tprev = c.tnext;
    } else {
        c.rejected++;
    }
    float tn = c.tprev + dtn;
    c.tprev = fminf(c.tprev, c.t1);
    if (tn > c.t1 - 1e-6f) tn = keep ? c.t1 : c.tprev + 0.5f * (c.t1 - c.tprev);
    c.tnext = tn;
    c.nsteps++;
    if (!(c.tprev < c.t1)) c.active = 0;
    if (c.active && c.nsteps >= p.max_steps) {
        c.flags |= 1;
        c.active = 0;
    }
}

// One diffeqsolve for the workgroup's envs (each wave drives its 2 envs'
// control; the coupling GEMM always covers all 16 rows).
template <int TPW>
__device__ void solve_wg(const DevParams& p, float* Xs, int* wg_flag, Ctl (&ctl)[ENVS_PER_WAVE], int env_base,
                         float (*smp_n)[KURA_S_MAX + 2], double (*smp_r)[KURA_S_MAX + 2], bool to_ring,
                         long long* rhs_count) {
    constexpr int EPL = TPW * 4;  // N / 64
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int N = p.N;
    floatx16 acc[TPW];
    // Y0 <- state y for active envs; initial RHS (stage 0)
#pragma unroll
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        const int env = env_base + wave * ENVS_PER_WAVE + ee;
        if (env >= p.B || !ctl[ee].active) continue;
#pragma unroll 4
        for (int m = 0; m < EPL; ++m) {
            const size_t o = (size_t)env * N + lane + 64 * m;
            p.Y0[o] = p.y[o];
        }
    }
    __syncthreads();
    stage_input<EPL>(p, Xs, ctl, env_base, 0);
    __syncthreads();
    coupling_gemm<TPW>(Xs, p.alpha_sw, N, acc);
    coupling_epilogue<TPW>(p, Xs, acc, env_base, 0);
    long long nrhs = 1;
    for (;;) {
        // workgroup-wide "any env still integrating?"
        __syncthreads();
        if (threadIdx.x == 0) *wg_flag = 0;
        __syncthreads();
        int mine = 0;
#pragma unroll
        for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) mine |= ctl[ee].active;
        if (mine && lane == 0) atomicOr(wg_flag, 1);
        __syncthreads();
        if (*wg_flag == 0) break;
#pragma unroll
        for (int ee = 0; ee < ENVS_PER_WAVE; ++ee)
            if (ctl[ee].active) ctl[ee].h = ctl[ee].tnext - ctl[ee].tprev;
        for (int s = 1; s <= 6; ++s) {
            stage_input<EPL>(p, Xs, ctl, env_base, s);
            __syncthreads();
            coupling_gemm<TPW>(Xs, p.alpha_sw, N, acc);
            coupling_epilogue<TPW>(p, Xs, acc, env_base, s);
            __syncthreads();
        }
        nrhs += 6;
#pragma unroll
        for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
            const int e = wave * ENVS_PER_WAVE + ee;
            const int env = env_base + e;
            if (env >= p.B || !ctl[ee].active) continue;
            double* rd = to_ring ? p.ring + (size_t)env * p.W : nullptr;
            post_step<EPL>(p, ctl[ee], env, smp_n[e], smp_r[e], rd);
        }
    }
    *rhs_count += nrhs;
}

__device__ __forceinline__ void ctl_begin(Ctl& c, const Grid& g, float dt0, int lfp_from, int lfp_to, int pos0) {
    c.g = g;
    const float t0 = (float)grid_at(g, 0);
    c.t1 = (float)grid_at(g, g.n - 1);
    c.tprev = t0;
    c.tnext = fminf(t0 + dt0, c.t1);
    c.h = 0.0f;
    c.si = 0;
    c.nsteps = 0;
    c.lfp_from = lfp_from;
    c.lfp_to = lfp_to;
    c.pos0 = pos0;
    c.active = g.n >= 2;
}

__device__ __forceinline__ void flush_stats(const DevParams& p, long long rhs, const Ctl (&ctl)[ENVS_PER_WAVE],
                                            int env_base) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane != 0) return;
    unsigned long long steps = 0, rej = 0, flags = 0;
#pragma unroll
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        if (env_base + wave * ENVS_PER_WAVE + ee >= p.B) continue;
        steps += ctl[ee].nsteps;
        rej += ctl[ee].rejected;
        flags |= ctl[ee].flags;
    }
    if (wave == 0) atomicMax(&p.stats[0], (unsigned long long)rhs);
    atomicAdd(&p.stats[1], steps);
    atomicAdd(&p.stats[2], rej);
    if (flags) atomicOr(&p.stats[3], flags);
}

// R64 dot of the window (lane-strided, registers) with a twiddle row.
template <int WPL>
__device__ __forceinline__ double window_dot(const double (&x)[WPL], const double* tab, int W) {
    const int lane = threadIdx.x & 63;
    double a = 0.0;
#pragma unroll
    for (int m = 0; m < WPL; ++m) {
        const int i = lane + 64 * m;
        if (i < W) a = __builtin_fma(x[m], tab[i], a);
    }
    return wave_sum_f64(a);
}

// R64 order replayed serially by one lane (used where a single lane owns the
// whole vector, e.g. the R2 filter output).
__device__ double serial_r64_f64(const double* v, int n) {
    double part[64];
    for (int l = 0; l < 64; ++l) {
        double a = 0.0;
        for (int i = l; i < n; i += 64) a = a + v[i];
        part[l] = a;
    }
    for (int o = 32; o >= 1; o >>= 1)
        for (int l = 0; l < 64; ++l)
            if (!(l & o)) {
                const double v = part[l] + part[l ^ o];  // == part[l^o] + part[l]
                part[l] = v;
                part[l ^ o] = v;
            }
    return part[0];
}

// Window accessor for the serial filter: x[i] (oldest first) is either an
// untouched slot of the ring or one of the S new samples held in LDS.
struct WinView {
    const double* ring;
    const double* fresh;
    int W, wp0, S;
    __device__ double at(int i) const {
        const int keep = W - S;
        if (i < keep) {
            int k = wp0 + S + i;
            if (k >= W) k -= W;
            return ring[k];
        }
        return fresh[i - keep];
    }
};

// R2 = -1e3 (filtfilt(x)[-1] - mean(filtfilt(x)))^2 - 1e-2|u0|, computed by
// lane 0 (scipy lfilter DF2T order, no contraction; oracle filtfilt_last_dev).
__device__ double filtfilt_last_dev(const DevParams& p, const WinView& xv, double* ext, double* tmp) {
    const int W = p.W, P = p.padlen, L = W + 2 * P;
    const double x0 = xv.at(0), xl = xv.at(W - 1);
    for (int i = 0; i < P; ++i) ext[i] = 2.0 * x0 - xv.at(P - i);
    for (int i = 0; i < W; ++i) ext[P + i] = xv.at(i);
    for (int i = 0; i < P; ++i) ext[P + W + i] = 2.0 * xl - xv.at(W - 2 - i);
    for (int pass = 0; pass < 2; ++pass) {
        const double e0 = ext[0];
        double z0 = p.bw_zi[0] * e0, z1 = p.bw_zi[1] * e0, z2 = p.bw_zi[2] * e0, z3 = p.bw_zi[3] * e0;
        for (int k = 0; k < L; ++k) {
            const double xn = ext[k];
            const double yn = z0 + p.bw_b[0] * xn;
            z0 = (z1 + xn * p.bw_b[1]) - yn * p.bw_a[1];
            z1 = (z2 + xn * p.bw_b[2]) - yn * p.bw_a[2];
            z2 = (z3 + xn * p.bw_b[3]) - yn * p.bw_a[3];
            z3 = xn * p.bw_b[4] - yn * p.bw_a[4];
            tmp[k] = yn;
        }
        if (pass == 0)
            for (int i = 0; i < L; ++i) ext[i] = tmp[L - 1 - i];
    }
    for (int i = 0; i < W; ++i) ext[i] = tmp[L - 1 - P - i];
    const double mean = serial_r64_f64(ext, W) / (double)W;
    return ext[W - 1] - mean;
}

// Reward of the window held in registers (R64 layout), env.py:638-688.
// Must be called by the whole wave (the DFT reductions shuffle).
template <int WPL>
__device__ double reward_of(const DevParams& p, const double (&x)[WPL], double u0, const WinView& xv, double* ext,
                            double* tmp) {
    const int lane = threadIdx.x & 63;
    const double au = fabs(u0);
    if (p.reward_kind == KURA_R_TEMP_CONST) {
        double r = 0.0;
        if (lane == 0) {
            const double d = filtfilt_last_dev(p, xv, ext, tmp);
            const double r1 = 1e3 * (d * d);
            r = -r1 - 1e-2 * au;
        }
        return __shfl(r, 0, 64);
    }
    double bb = 0.0;
    for (int b = 0; b < p.n_bins; ++b) {
        const double re = window_dot<WPL>(x, p.ctab + (size_t)b * p.W, p.W);
        const double im = window_dot<WPL>(x, p.stab + (size_t)b * p.W, p.W);
        const double pr = re / (double)p.W, pi = im / (double)p.W;
        const double pw = (pr * pr + pi * pi) * 2.0;
        bb = bb + pw;
    }
    if (p.reward_kind == KURA_R_BBPOW_THR) {
        const double bs = 1e4 * bb;
        const double r1 = bs > 20.0 ? 5.0 : 0.0;
        return -r1 - au;
    }
    const double r1 = 1e4 * bb;
    return -r1 - 1e-2 * au;
}

#define WPL_MAX 40  // ceil(W/64) upper bound supported (W <= 2560)

// ------------------------------------------------------------ step kernel --
template <int TPW>
__global__ __launch_bounds__(NTHREADS) void kura_step_kernel(DevParams p, const float* __restrict__ action,
                                                             float* __restrict__ obs, double* __restrict__ reward,
                                                             uint8_t* __restrict__ done, float* __restrict__ lfp_true,
                                                             double* __restrict__ lfp_rec, int* __restrict__ nsamp) {
    extern __shared__ float Xs[];  // 32 * N floats
    __shared__ float smp_n[E_WG][KURA_S_MAX + 2];
    __shared__ double smp_r[E_WG][KURA_S_MAX + 2];
    __shared__ int wg_flag;
    constexpr int EPL = TPW * 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int N = p.N;
    const int env_base = blockIdx.x * E_WG;
    Ctl ctl[ENVS_PER_WAVE];
    double u0v[ENVS_PER_WAVE];
    int nI[ENVS_PER_WAVE], nII[ENVS_PER_WAVE], steps[ENVS_PER_WAVE], rej[ENVS_PER_WAVE], flg[ENVS_PER_WAVE];
    // ---- stimulation ON: pulse = float32(sum_e g_e * u_e)  (env.py:419-424)
#pragma unroll
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        const int env = env_base + wave * ENVS_PER_WAVE + ee;
        ctl[ee].active = 0;
        ctl[ee].rejected = 0;
        ctl[ee].flags = 0;
        ctl[ee].nsteps = 0;
        nI[ee] = 0;
        nII[ee] = 0;
        u0v[ee] = 0.0;
        if (env >= p.B) continue;
        double u[4] = {0.0, 0.0, 0.0, 0.0};
        const int ne = p.n_elec < 4 ? p.n_elec : 4;
        for (int e = 0; e < ne; ++e) {
            const double a = (double)action[(size_t)env * p.n_elec + e];
            u[e] = p.dbs_lo + ((p.dbs_hi - p.dbs_lo) * (a - p.act_lo)) / (p.act_hi - p.act_lo);
        }
        u0v[ee] = u[0];
        for (int m = 0; m < EPL; ++m) {
            const int i = lane + 64 * m;
            double pacc = 0.0;
            for (int e = 0; e < ne; ++e) pacc = pacc + p.g_stim[((size_t)env * p.n_elec + e) * N + i] * u[e];
            p.pulse[(size_t)env * N + i] = (float)pacc;
        }
        const double t = p.t[env];
        const Grid g = make_grid(t, t + p.width, p.dt);
        nI[ee] = g.n;
        ctl_begin(ctl[ee], g, p.dt0, 0, g.n, 0);
        if (g.n < 2 || g.n > KURA_S_MAX) {
            ctl[ee].active = 0;
            ctl[ee].flags |= 8;
        }
    }
    long long rhs = 0;
    solve_wg<TPW>(p, Xs, &wg_flag, ctl, env_base, smp_n, smp_r, false, &rhs);
    // ---- stimulation OFF (env.py:433-441)
#pragma unroll
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        const int e = wave * ENVS_PER_WAVE + ee;
        const int env = env_base + e;
        steps[ee] = ctl[ee].nsteps;
        rej[ee] = ctl[ee].rejected;
        flg[ee] = ctl[ee].flags;
        ctl[ee].active = 0;
        if (env >= p.B || flg[ee]) continue;
        for (int m = 0; m < EPL; ++m) p.pulse[(size_t)env * N + lane + 64 * m] = 0.0f;
        const double tm = grid_at(ctl[ee].g, nI[ee] - 1);
        const Grid g = make_grid(tm, tm + p.pause, p.dt);
        nII[ee] = g.n;
        ctl_begin(ctl[ee], g, p.dt0, 1, g.n - 1, nI[ee] + 1);
        ctl[ee].rejected = 0;
        ctl[ee].flags = 0;
        if (g.n < 2 || nI[ee] + g.n - 1 > KURA_S_MAX) {
            ctl[ee].active = 0;
            flg[ee] |= 8;
        }
        if (lane == 0) {  // ys_II[0] == ys_I[-1]: duplicated sample (env.py:440)
            smp_n[e][nI[ee]] = smp_n[e][nI[ee] - 1];
            smp_r[e][nI[ee]] = smp_r[e][nI[ee] - 1];
        }
    }
    solve_wg<TPW>(p, Xs, &wg_flag, ctl, env_base, smp_n, smp_r, false, &rhs);
    __syncthreads();
    // ---- window, reward, outputs (env.py:443-454)
    constexpr int WPL = WPL_MAX;
#pragma unroll 1
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        const int e = wave * ENVS_PER_WAVE + ee;
        const int env = env_base + e;
        steps[ee] += ctl[ee].nsteps;
        rej[ee] += ctl[ee].rejected;
        flg[ee] |= ctl[ee].flags;
        ctl[ee].nsteps = steps[ee];
        ctl[ee].rejected = rej[ee];
        ctl[ee].flags = flg[ee];
        if (env >= p.B) continue;
        const int S = nI[ee] + nII[ee] - 1;
        if (flg[ee] || S < 1) {
            if (lane == 0) {
                if (nsamp) nsamp[env] = 0;
                if (done) done[env] = 1;
                if (reward) reward[env] = 0.0;
            }
            continue;
        }
        const int W = p.W;
        double* rb = p.ring + (size_t)env * W;
        const int wp0 = p.wpos[env];
        const WinView xv{rb, &smp_r[e][0], W, wp0, S};
        double x[WPL];
#pragma unroll
        for (int m = 0; m < WPL; ++m) {
            const int i = lane + 64 * m;
            x[m] = 0.0;
            if (i < W) {
                x[m] = xv.at(i);
                if (obs) obs[(size_t)env * W + i] = (float)x[m];
            }
        }
        double* ext = p.scratch + (size_t)env * 2 * (W + 2 * p.padlen);
        double* tmp = ext + (W + 2 * p.padlen);
        const double r = reward_of<WPL>(p, x, u0v[ee], xv, ext, tmp);
        // ring append after every read of the old slots
        if (lane < S) {
            int k = wp0 + lane;
            if (k >= W) k -= W;
            rb[k] = smp_r[e][lane];
        }
        int wp = wp0 + S;
        if (wp >= W) wp -= W;
        if (lane == 0) {
            p.wpos[env] = wp;
            const int st = p.step[env] + 1;
            p.step[env] = st;
            p.t[env] = grid_at(ctl[ee].g, nII[ee] - 1);
            if (reward) reward[env] = r;
            if (done) done[env] = st >= p.episode_steps;
            if (nsamp) nsamp[env] = S;
        }
        if (lane < KURA_S_MAX) {
            if (lfp_true) lfp_true[(size_t)env * KURA_S_MAX + lane] = lane < S ? smp_n[e][lane] : 0.0f;
            if (lfp_rec) lfp_rec[(size_t)env * KURA_S_MAX + lane] = lane < S ? smp_r[e][lane] : 0.0;
        }
    }
    flush_stats(p, rhs, ctl, env_base);
}

// ----------------------------------------------------------- reset kernel --
template <int TPW>
__global__ __launch_bounds__(NTHREADS) void kura_reset_kernel(DevParams p, const uint8_t* __restrict__ mask,
                                                              const float* __restrict__ theta0,
                                                              float* __restrict__ obs) {
    extern __shared__ float Xs[];
    __shared__ float smp_n[E_WG][KURA_S_MAX + 2];
    __shared__ double smp_r[E_WG][KURA_S_MAX + 2];
    __shared__ int wg_flag;
    constexpr int EPL = TPW * 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int N = p.N, W = p.W;
    const int env_base = blockIdx.x * E_WG;
    Ctl ctl[ENVS_PER_WAVE];
#pragma unroll
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        const int env = env_base + wave * ENVS_PER_WAVE + ee;
        ctl[ee].active = 0;
        ctl[ee].rejected = 0;
        ctl[ee].flags = 0;
        ctl[ee].nsteps = 0;
        if (env >= p.B || (mask && !mask[env])) continue;
        for (int m = 0; m < EPL; ++m) {
            const size_t o = (size_t)env * N + lane + 64 * m;
            p.y[o] = theta0[o];
            p.pulse[o] = 0.0f;
        }
        const Grid g = make_grid(0.0, p.transient_len, p.dt);
        ctl_begin(ctl[ee], g, p.dt0, g.n - 1 - W, g.n - 1, 0);
    }
    long long rhs = 0;
    solve_wg<TPW>(p, Xs, &wg_flag, ctl, env_base, smp_n, smp_r, true, &rhs);
    __syncthreads();
#pragma unroll
    for (int ee = 0; ee < ENVS_PER_WAVE; ++ee) {
        const int env = env_base + wave * ENVS_PER_WAVE + ee;
        if (env >= p.B || (mask && !mask[env])) continue;
        if (lane == 0) {
            p.t[env] = grid_at(ctl[ee].g, ctl[ee].g.n - 1);
            p.step[env] = 0;
            p.wpos[env] = 0;
        }
        if (obs)
            for (int i = lane; i < W; i += 64) obs[(size_t)env * W + i] = (float)p.ring[(size_t)env * W + i];
    }
    flush_stats(p, rhs, ctl, env_base);
}

// ------------------------------------------------------ standalone reward --
template <int WPL>
__global__ __launch_bounds__(64) void kura_reward_kernel(DevParams p, const double* __restrict__ win,
                                                         const float* __restrict__ u0, double* __restrict__ out,
                                                         int n) {
    const int env = blockIdx.x;
    if (env >= n) return;
    const int lane = threadIdx.x;
    const double* xl = win + (size_t)env * p.W;
    double x[WPL];
#pragma unroll
    for (int m = 0; m < WPL; ++m) {
        const int i = lane + 64 * m;
        x[m] = i < p.W ? xl[i] : 0.0;
    }
    double* ext = p.scratch + (size_t)p.B * 2 * (p.W + 2 * p.padlen) + (size_t)env * 2 * (p.W + 2 * p.padlen);
    double* tmp = ext + (p.W + 2 * p.padlen);
    const WinView xv{xl, xl, p.W, 0, 0};
    const double r = reward_of<WPL>(p, x, (double)u0[env], xv, ext, tmp);
    if (lane == 0) out[env] = r;
}

// ------------------------------------------------------------- self-tests --
__global__ void kura_selftest_math_kernel(const float* x, const float* y, float* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s, c;
    kdm_sincosf(x[i], &s, &c);
    out[(size_t)i * 8 + 0] = s;
    out[(size_t)i * 8 + 1] = c;
    out[(size_t)i * 8 + 2] = kdm_fmod2pi(x[i]);
    out[(size_t)i * 8 + 3] = kdm_inv_fifth_root(fabsf(y[i]));
    out[(size_t)i * 8 + 4] = sqrtf(fabsf(x[i]));
    out[(size_t)i * 8 + 5] = x[i] / y[i];
    out[(size_t)i * 8 + 6] = (float)((double)x[i] / (double)y[i]);
    out[(size_t)i * 8 + 7] = (float)ceil((double)x[i] / 0.05);
}

// One 32-row coupling GEMM through the production GEMM path.
template <int TPW>
__global__ __launch_bounds__(NTHREADS) void kura_selftest_gemm_kernel(const float* X, const float* alpha_sw,
                                                                       float* Y, int N) {
    extern __shared__ float Xs[];
    for (int idx = threadIdx.x; idx < 32 * N; idx += blockDim.x) {
        const int r = idx / N, k = idx % N;
        Xs[xs_idx(r, k)] = X[idx];
    }
    __syncthreads();
    floatx16 acc[TPW];
    coupling_gemm<TPW>(Xs, alpha_sw, N, acc);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
            const int col = 32 * (wave * TPW + t) + (lane & 31);
            Y[(size_t)row * N + col] = acc[t][q];
        }
}

// explicit instantiations are made by the launchers in kura_capi.hip
#include "kura_capi.inc"
