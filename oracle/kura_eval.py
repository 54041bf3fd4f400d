"""CPU restatement of the reference's episode evaluation metric -- TEST
INFRASTRUCTURE (only tests/ may import it; the product computes the metric in
libkura's kura_psd_kernel).

calc_psd_for_simple_eval(sig_envs, psd_dt, beta_a=12.5, beta_b=21) follows
aDBS_RL/evaluate_HF_DBS.py:122-135 and band_pass_envelope
environment/utils.py:794-816 (order=2 as called there; the Hilbert envelope is
computed by the reference but unused by the metric).  Pinned against the
reference function itself: tests/golden/make_golden_eval.py.
"""
from __future__ import annotations

import numpy as np
from scipy.signal import butter, filtfilt


def band_pass(sig, fs, lowcut=12.0, highcut=30.0, order=2):
    nyq = 0.5 * fs
    b, a = butter(order, [lowcut / nyq, highcut / nyq], btype="band")
    return filtfilt(b, a, sig)


def calc_psd_for_simple_eval(sig_envs, psd_dt, beta_a=12.5, beta_b=21.0):
    out = []
    for sig in sig_envs:
        sf = band_pass(np.asarray(sig), 1.0 / psd_dt)
        ft = np.abs(np.fft.rfft(sf) / sf.shape[0]) ** 2 * 2
        freq = np.fft.rfftfreq(sf.shape[0], psd_dt)
        ft = filtfilt([1] * 12, 5, ft)
        idx = np.where((freq > beta_a) & (freq < beta_b))
        out.append(np.sum(ft[idx]))
    return np.asarray(out)


def envelope_stats(sig_envs):
    """log_main_metrics('per_episode', 'envelope', calc_envelope(lfp_ep))
    (aDBS_RL/agents/custom_callbacks.py:146-148, :28-31) in float64:
    calc_envelope = |scipy.signal.hilbert(x)| (environment/utils.py:835-836),
    restated as scipy defines it -- X = fft(x); X[1:n/2] *= 2 (and X[n/2] kept
    for even n); negative bins zeroed; |ifft(X)|.  Returns [n, 3] = mean,
    std(ddof=1) (NaN for one sample), sum.  The reference runs this in
    complex64 for float32 input; pinned to it at 1e-5 relative
    (tests/golden/make_golden_envelope.py)."""
    out = []
    for sig in sig_envs:
        x = np.asarray(sig, np.float64)
        n = x.shape[0]
        X = np.fft.fft(x)
        h = np.zeros(n)
        h[0] = 1.0
        if n % 2 == 0:
            h[n // 2] = 1.0
            h[1:n // 2] = 2.0
        else:
            h[1:(n + 1) // 2] = 2.0
        e = np.abs(np.fft.ifft(X * h))
        sd = float(np.std(e, ddof=1)) if n > 1 else float("nan")
        out.append([float(np.mean(e)), sd, float(np.sum(e))])
    return np.asarray(out, np.float64)
