/*
 * kura.h -- C ABI of libkura, the MI355X-native batched Kuramoto simulator
 * that replaces SpatialKuramoto.step()/reset() of the reference
 * (environment/env.py:415-454 and :467-614).
 *
 * One handle owns B independent environments on one GPU.  All per-step I/O
 * pointers are DEVICE pointers allocated by the caller (PyTorch-ROCm tensors
 * via tensor.data_ptr()); they are borrowed for the duration of the call and
 * the work is enqueued on the given hipStream_t (NULL = default stream).
 * Setup calls take HOST pointers and are synchronous.  kura_step and
 * kura_reset never allocate device memory (kura_create does it once); the
 * episode-metric calls grow a per-handle scratch on demand and kura_reward_n
 * builds (synchronously, once per window length) the R2 filter functional of
 * that length, keeping those of the 4 most recently used lengths (a fifth
 * length synchronises the device and frees the least recently used).  Errors
 * never throw across the ABI: every
 * call returns 0 on success or a negative KURA_E* code, and
 * kura_last_error() returns a thread-local message.
 *
 * Reference interfaces each entry point replaces (file:line under the
 * reference tree):
 *   kura_create          SpatialKuramoto.__init__        env.py:277-386
 *   kura_set_coupling    KuramotoJAX.__init__ alpha     env.py:219-229
 *   kura_set_env_params  apply_locus_mask + SimpleDBS    env.py:566-593, :61-156
 *   kura_set_env_gain    KuramotoJAX(K=...) per env      env.py:264, :570-593
 *   kura_set_spectral    calc_beta_band_power bins       utils.py:21-27
 *   kura_reset           SpatialKuramoto.reset transient env.py:594-614
 *   kura_step            SpatialKuramoto.step            env.py:415-454
 *   kura_reward          reward_* on a given window      env.py:638-688
 *   kura_reward_n        reward_* on any window length   env.py:638-688, utils.py:21-27
 *   kura_get/set_state   (no reference equivalent; env state was not
 *   kura_get/set_spec    checkpointable)
 *
 * Rewards (env.py:638-688) inside kura_step: R2's filtfilt term is the dot
 * product c . x of the window with the filter's linear functional c
 * (filtfilt(x)[-1] - mean(filtfilt(x)) is linear in x; dbs-gym_amd/csrc/
 * kura_r2.h builds c once per handle); R1/R3's beta bins come from running
 * spectral accumulators Y_k = sum_p ring[p] e^{-2 pi i k p/W} over ring
 * positions, updated by the S slots each step overwrites (|X_k| = |Y_k|).
 * Both agree with scipy / numpy's rfft to float64 rounding.
 */
#ifndef KURA_H
#define KURA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.  1: rounds 1-4.  2: KuraConfig.coupling takes the former
 * reserved_i[0] slot (0 = AUTO, which resolves to BF16X3: a zero-filled
 * version-1 config would silently change arithmetic, so kura_create rejects
 * abi_version 1), kura_set_transient_capture, kura_selftest_coupling. */
#define KURA_ABI_VERSION 2
#define KURA_S_MAX 32   /* max LFP samples emitted by one step (ref: 17-19) */
#define KURA_MAX_BINS 32

enum {
    KURA_OK = 0,
    KURA_E_INVALID = -1,   /* bad argument (ref: ValueError/AssertionError) */
    KURA_E_HIP = -2,       /* HIP runtime error */
    KURA_E_NOMEM = -3,
    KURA_E_UNSUPPORTED = -4,
    KURA_E_STATE = -5      /* call order violated (e.g. step before reset) */
};

/* per-env failure bits of a step/reset launch (kura_get_env_flags, and OR-ed
 * over the launch into kura_get_stats()[3]).  The reference's diffeqsolve
 * raises on a failed solve (diffrax throw=True, env.py:261-270); libkura never
 * throws: a failed env's step is abandoned (done = 1, reward = 0, nsamp = 0,
 * obs/lfp/window/time/step counter not written) and the host decides.  The
 * env's phase state is then UNDEFINED -- if the stim-ON solve succeeded and
 * the stim-OFF solve failed, y already holds the ON solve's last row (the
 * oracle behaves the same way) -- so a failed env must be reset
 * (KuraVectorEnv does this for on_failure="reset"); a failed reset likewise
 * leaves t at the end of the transient with an undefined y. */
enum {
    KURA_F_MAX_STEPS = 1,   /* diffeqsolve max_steps reached */
    KURA_F_NONFINITE = 2,   /* NaN/Inf state or RHS (non-finite error norm) */
    KURA_F_GRID = 8,        /* save grid outside [2, KURA_S_MAX] samples */
    KURA_F_BARRIER = 16,    /* split-group (N > 1024) barrier timed out: every
                               exchange after it is unsynchronised */
    KURA_F_BOUNDS = 32      /* KURA_DEBUG builds (libkura_debug.so) only: a
                               record / alpha / ring / sample access outside
                               its buffer (kura_get_stats()[3]) */
};

enum { KURA_REC_NAIVE = 0, KURA_REC_GAUSSIAN = 1 };             /* env.py:333-338 */

/* Coupling arithmetic (KuraConfig.coupling).  Both are exact, deterministic
 * restatements of the reference's fp32 sum (env.py:252-256, JAX x64 off) with
 * different last-bit rounding; both agree with the reference's own op
 * sequence to <= 5e-7 absolute per RHS (tests/test_golden_reference.py):
 *   F32     every product and sum in fp32: a k-ordered fmaf chain from +0
 *           (v_mfma_f32_32x32x2_f32 computes exactly that);
 *   BF16X3  each fp32 operand split into three bf16 parts (x = x1 + x2 + x3,
 *           round-to-nearest-even, exact residuals), the six products
 *           x1a1, x1a2, x2a1, x1a3, x2a2, x3a1 per 16-deep k-block on
 *           v_mfma_f32_32x32x16_bf16 with fp32 accumulation (the oracle
 *           restates that MFMA's accumulation exactly); ~1.4x the F32 rate
 *           at n_osc <= 1024; any n_osc (split env groups included);
 *   AUTO    BF16X3 at every n_osc (split env groups included: 1.2-1.4x F32
 *           there, and within the same 5e-7 of the reference RHS at
 *           n_osc = 8192, tests/test_golden_reference.py). */
enum { KURA_COUPLING_AUTO = 0, KURA_COUPLING_F32 = 1, KURA_COUPLING_BF16X3 = 2 };
/* kura_coupling_of(cfg), below: the arithmetic a config resolves to (the
 * library and the oracle share it) */
enum { KURA_R_BBPOW = 1, KURA_R_TEMP_CONST = 2, KURA_R_BBPOW_THR = 3 }; /* env.py:323-330 */

typedef struct KuraConfig {
    int32_t abi_version;   /* must be KURA_ABI_VERSION */
    int32_t n_osc;         /* N, params_dict['num_oscillators'] */
    int32_t n_envs;        /* B, environments in this handle */
    int32_t window;        /* W = int(step_len*observe_wind_counts/verbose_dt), env.py:294-297;
                              KURA_S_MAX <= W <= 2560 */
    int32_t n_elec;        /* stimulating contacts = len(elec_coords), env.py:93-95 */
    int32_t n_rec;         /* recording contacts = len(rec_coords), env.py:96-98 */
    int32_t rec_kernel;    /* KURA_REC_* */
    int32_t reward_kind;   /* KURA_R_* */
    int32_t episode_steps; /* total_episode_counts, env.py:300 */
    int32_t max_steps;     /* diffrax diffeqsolve max_steps default (4096) */
    int32_t n_bins;        /* rfft bins with beta_a < f < beta_b (utils.py:24-26) */
    int32_t bins[KURA_MAX_BINS];
    int32_t padlen;        /* filtfilt padlen for R2 (3*max(len(a),len(b)) = 15) */
    int32_t episode_cap;   /* >0: keep each env's true-LFP samples of the running episode (up to this
                              many) for kura_episode_bbpow (evaluate_HF_DBS.py:83,122-135); 0: off */
    int32_t part_osc;      /* N > 1024 (split env groups): oscillators per workgroup, 256, 512 or 1024
                              (0 = 1024); smaller parts put more workgroups on the chip when the
                              handle has few envs.  It fixes the solver's reduction order (the
                              oracle follows it), so results depend on it bit for bit. */
    int32_t coupling;      /* KURA_COUPLING_*: the arithmetic of the O(N^2) coupling sums
                              P = alpha.sin(theta), Q = alpha.cos(theta) of every RHS
                              (env.py:252-256); results depend on it bit for bit, and the
                              oracle follows it (kura_coupling_of) */
    int32_t reserved_i[1];
    double dt;             /* verbose_dt: save-grid spacing (units) */
    double width;          /* electrode_width: stimulation ON interval */
    double pause;          /* electrode_pause: OFF interval */
    double transient_len;  /* transient_state_len */
    double act_lo, act_hi; /* ppo_action_bounds  [-1, 1]  env.py:309 */
    double dbs_lo, dbs_hi; /* dbs_action_bounds  [-5, 5]  env.py:308 */
    double bw_b[5];        /* butter(2, [12, 30]/(fs/2), 'band') numerator  (utils.py:812) */
    double bw_a[5];        /* ... denominator */
    double bw_zi[4];       /* scipy.signal.lfilter_zi(b, a) */
    double reserved_d[4];
    float rtol, atol;      /* PIDController(rtol=1e-5, atol=1e-5), env.py:249 */
    float kn;              /* float32(K / N), env.py:264 */
    float dt0;             /* diffeqsolve dt0 = 0.05, env.py:267 */
    float reserved_f[4];
} KuraConfig;

static inline int kura_coupling_of(const struct KuraConfig* c) {
    if (c->coupling == KURA_COUPLING_AUTO) return KURA_COUPLING_BF16X3;
    return c->coupling;
}

typedef struct KuraHandle KuraHandle;

/* create / destroy */
int kura_create(const KuraConfig* cfg, int device, KuraHandle** out);
int kura_destroy(KuraHandle* h);
const char* kura_last_error(void);
int kura_abi_version(void);

/* setup (host pointers, synchronous) */
int kura_set_coupling(KuraHandle* h, const float* alpha /* N*N row-major, alpha[i][j] */);
int kura_set_env_params(KuraHandle* h, int env0, int n,
                        const float* omega,   /* n*N  (float32 cast of w0, env.py:264) */
                        const double* g_stim, /* n*n_elec*N conductances, env.py:106-120 */
                        const double* g_rec); /* n*n_rec*N  recorder conductances, :142-156 */
/* calc_psd_for_simple_eval (aDBS_RL/evaluate_HF_DBS.py:122-135) of n device
 * signals sig[j*ld ...] of len[j] float32 samples (an episode's concatenated
 * true LFP): band_pass_envelope filtfilt (butter(2, [12,30]/(fs/2))), |rfft/n|^2*2,
 * filtfilt(ones(12), 5, .) smoothing of the whole half spectrum, sum over
 * beta_a < f < beta_b with f = k/(len*psd_dt).  Any length and band: the
 * spectrum is a Bluestein DFT (power-of-two FFTs of 2^m >= 2*len-1 points).
 * out[j] (device f64) is NaN for len[j] < 72, where the reference raises
 * (scipy filtfilt needs len/2+1 > padlen = 36).  Float64 throughout; agrees
 * with NumPy/SciPy to ~1e-12 relative (not bitwise: different FFT).
 * All metric calls on one handle share its scratch buffer: issue them on one
 * stream (growing the buffer synchronises the device). */
int kura_psd_bbpow(KuraHandle* h, const float* sig, const int32_t* len, int64_t ld, int n, double psd_dt,
                   double beta_a, double beta_b, double* out, void* stream);
/* the same metric of every env's current-episode true LFP (requires
 * cfg.episode_cap > 0); mask[b] (device, NULL = all) selects envs; out[b]
 * NaN for unselected envs and for episodes longer than episode_cap.  Call it
 * after the last kura_step of an episode and before the kura_reset that
 * starts the next one (KuraVectorEnv does so for autoreset envs). */
int kura_episode_bbpow(KuraHandle* h, const uint8_t* mask, double psd_dt, double beta_a, double beta_b,
                       double* out, void* stream);
/* per-episode envelope statistics of the training callback
 * (aDBS_RL/agents/custom_callbacks.py:146-148: log_main_metrics('per_episode',
 * 'envelope', calc_envelope(lfp_ep)), with calc_envelope = |hilbert(x)|,
 * environment/utils.py:835-836, and log_main_metrics = mean, std(ddof=1),
 * sum, custom_callbacks.py:28-31) of n device signals sig[j*ld ...] of len[j]
 * float32 samples.  out[3j..3j+2] (device f64) = mean, std, sum; NaN for
 * len[j] outside [1, ld] (std NaN for len 1).  Float64 Bluestein DFTs
 * (O(len log len)); SciPy's hilbert of float32 input runs in complex64, so
 * the reference agrees to ~1e-5 relative, the float64 restatement to ~1e-10. */
int kura_envelope_stats(KuraHandle* h, const float* sig, const int32_t* len, int64_t ld, int n, double* out,
                        void* stream);
/* the same statistics of every env's current-episode true LFP (requires
 * cfg.episode_cap > 0); mask[b] (device, NULL = all) selects envs; out[3b..]
 * NaN for unselected envs.  Call it where kura_episode_bbpow is called. */
int kura_episode_envelope_stats(KuraHandle* h, const uint8_t* mask, double* out, void* stream);
/* per-env coupling gain float32(K_b / N) for envs [env0, env0+n) (host
 * array; each reference env has its own params_dict['K'], env.py:264).  Envs
 * not set keep the config's kn. */
int kura_set_env_gain(KuraHandle* h, int env0, int n, const float* kn);
int kura_set_spectral(KuraHandle* h, const double* cos_tab, const double* sin_tab /* n_bins*W */);

/* hot path (device pointers, asynchronous on stream) */
int kura_reset(KuraHandle* h, const uint8_t* mask /* B or NULL = all */,
               const float* theta0 /* B*N float32 initial phases */,
               float* obs /* B*W or NULL */, void* stream);
int kura_step(KuraHandle* h, const float* action /* B*n_elec in [-1,1] */,
              float* obs,       /* B*W   float32 window, oldest first */
              double* reward,   /* B     */
              uint8_t* done,    /* B     */
              float* lfp_true,  /* B*KURA_S_MAX  theta_mean (naive LFP), env.py:444 */
              double* lfp_rec,  /* B*KURA_S_MAX  theta_records, env.py:445 (may be NULL) */
              int32_t* nsamp,   /* B     samples emitted this step (17..19) */
              void* stream);
/* reward of n given windows (oldest first) with first amplitudes u0 (already
 * rescaled, env.py:419); kind = KURA_R_* or 0 for the handle's reward_kind
 * (R1/R3 as direct float64 DFT dots of the window, R2 as c . x).
 * The reference exposes all three reward methods on every env (called
 * directly by aDBS_RL/agents/simple_dbs.py:83-90). */
int kura_reward(KuraHandle* h, int kind, const double* window /* n*W device */, const float* u0 /* n device */,
                double* reward /* n device */, int n, void* stream);
/* the same on 1-D windows of ANY length len (row stride ld >= len, device):
 * the reference's reward_* take the beta bins from len(x_state)
 * (env.py:638-688 -> utils.py:21-27; e.g. PIDController.predict passes
 * observation.ravel(), n_envs*W samples, aDBS_RL/agents/simple_dbs.py:81-88).
 * cos_tab/sin_tab: n_bins rows of len twiddles cos/sin(2 pi k i / len) for
 * the in-band bins k (device; unused for KURA_R_TEMP_CONST, which requires
 * len > padlen as scipy.signal.filtfilt does and uses the length-len filter
 * functional).  A call with len == W and the handle's tables equals
 * kura_reward bit for bit. */
int kura_reward_n(KuraHandle* h, int kind, const double* x /* n*ld device */, int64_t len, int64_t ld, int n,
                  const double* cos_tab, const double* sin_tab, int n_bins, const double* u0 /* n device, float64 */,
                  double* reward /* n device */, void* stream);

/* state snapshot for checkpoint/resume and parity tests (host pointers; syncs) */
int kura_get_state(KuraHandle* h, float* y /* B*N */, double* t /* B */, int32_t* step /* B */,
                   double* ring /* B*W */, int32_t* wpos /* B */);
int kura_set_state(KuraHandle* h, const float* y, const double* t, const int32_t* step,
                   const double* ring, const int32_t* wpos);
/* R1/R3 spectral accumulators (B * 2 * n_bins float64: re, im of each in-band
 * bin per env; host pointers; syncs).  kura_reset forms them from the new
 * window and kura_step updates them; kura_set_state (with a ring) and
 * kura_set_spectral re-form them from the ring, which equals the running
 * values to float64 rounding -- kura_set_spec restores a checkpoint's values
 * exactly (NULL: re-form from the ring). */
int kura_get_spec(KuraHandle* h, double* out);
int kura_set_spec(KuraHandle* h, const double* in);
#ifdef KURA_DEBUG
/* KURA_DEBUG builds (libkura_debug.so) only, not exported by libkura.so:
 * copy the solver workspace (records, [B_pad/16][14][N][16] float32, B_pad =
 * B rounded up to 16; syncs) to the host -- used to compare kernel
 * generations record by record (tools/record_probe.py) */
int kura_debug_read_workspace(KuraHandle* h, float* out, int64_t n);
/* ... and keep the sin/cos operand and the coupling sums of the first n RHS
 * sweeps of workgroup 0 (N <= 1024) in dev_buf ([n][2][32][N] float32, device;
 * NULL stops) -- tools/coupling_dump_probe.py */
int kura_debug_gemm_dump(KuraHandle* h, float* dev_buf, int n);
#endif
/* optional capture of every saved phase row of each kura_step: rows_dev
 * (device, B*(KURA_S_MAX+1)*N float32, or NULL to stop) receives, per env,
 * rows 0 .. S of the step -- ys_I then ys_II, the reference's sol_state_
 * (env.py:430,440; S = nsamp, row S is the new state).  Costs one extra
 * store per saved value; off by default. */
int kura_set_row_capture(KuraHandle* h, float* rows_dev);

/* optional record of a reset's transient (env.py:610-611,
 * theta_record_transient = calc_lfp(sol_state[:-1])): lfp_dev (device,
 * B*(T-1) float64 with T = len(np.arange(0, transient_state_len,
 * verbose_dt)), or NULL to stop) receives, for each env a kura_reset
 * resets, the LFP of every transient row but the last (the last W of them
 * are the observation window).  Costs the LFP of T-1-W more rows per
 * reset; off by default. */
int kura_set_transient_capture(KuraHandle* h, double* lfp_dev);

/* optional record of a reset's transient rows (env.py:610, sol_state =
 * kuramoto.forward(t_eval_transient, init_state), read after reset()):
 * rows_dev (device, B*T*N float32, T = kura_transient_len(h) =
 * len(np.arange(0, transient_state_len, verbose_dt)), or NULL to stop)
 * receives, for each env a kura_reset resets, every saved row of the
 * transient, row T-1 being the new state.  Every row is then evaluated (as
 * with kura_set_transient_capture) plus one store per value; off by
 * default.  T*N*4 bytes per env: 16 MB at N=1024 -- meant for a few envs. */
int kura_set_transient_rows(KuraHandle* h, float* rows_dev);
int kura_transient_len(KuraHandle* h);   /* T above (> 0), or a negative KURA_E_* */

/* per-env KURA_F_* bits of the last kura_step / kura_reset (0 = ok), copied
 * into the caller's device buffer out_dev (B int32) on the given stream:
 * read them with the step's outputs (no extra synchronisation). */
int kura_get_env_flags(KuraHandle* h, int32_t* out_dev, void* stream);

/* counters (synchronises the device), first min(n, KURA_NSTATS) written:
 * last call:  [0] RHS sweeps issued by the busiest workgroup, [1] Dopri5 steps
 *             attempted (all envs), [2] rejected, [3] KURA_F_* bits OR-ed over
 *             the envs, [4] RHS sweeps issued summed over
 *             workgroups (each sweep covers 16 env slots);
 * since kura_create: [5] steps attempted, [6] workgroup sweeps, [7] rejected. */
#define KURA_NSTATS 8
int kura_get_stats(KuraHandle* h, int64_t* out, int n);

/* diagnostics for the GPU parity tests (host pointers; synchronous; not on
 * the step path).  selftest_math writes 10 floats per element: sin, cos,
 * fmod2pi, inv_fifth_root(|y|), sqrt(|x|), x/y, f32(f64 x / f64 y),
 * ceil(x/0.05), and sin, cos of fmod(x, 2pi_f) (the RHS's folded reduction).  selftest_gemm runs the production MFMA coupling GEMM on one
 * 32 x N operand: Y[r][i] = sum_k X[r][k] * alpha[i][k] (N in {256, 512, 1024}). */
int kura_selftest_math(const float* x, const float* y, float* out, int n);
int kura_selftest_gemm(const float* X, const float* alpha, float* Y, int N);   /* KURA_COUPLING_F32 */
/* the same through the GEMM of a coupling arithmetic (KURA_COUPLING_*; AUTO = BF16X3 at these N) */
int kura_selftest_coupling(const float* X, const float* alpha, float* Y, int N, int coupling);
/* per-wave phase cycle counters of a -DKURA_STAMPS build ([8 waves][16]:
 * stage-input, barrier, GEMM, epilogue, barrier, post-step error pass, flag,
 * post-step decision, saves, FSAL, time advance, 5 spare; tools/phase_stamps.py);
 * zeros in the production build.  Reading clears them. */
int kura_get_stamps(KuraHandle* h, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* KURA_H */
