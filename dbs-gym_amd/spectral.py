"""Reward-side constants computed once on the host.

* beta-band rfft bins of calc_beta_band_power (utils.py:21-27) for the
  window length W and psd_dt = units2sec(verbose_dt) (env.py:647);
* the DFT twiddle tables the device uses for those bins (fp64);
* the order-2 Butterworth band-pass of band_pass_envelope (utils.py:794-816)
  and its lfilter_zi, for reward R2 (env.py:653-666).
"""
from __future__ import annotations

import numpy as np
from scipy.signal import butter, lfilter_zi

BETA_BAND = (12.5, 21.0)  # env.py:644, :677


def units2sec(x):
    """utils.py:830-832: 1 unit = 10 ms."""
    return x / 100


def beta_bins(W: int, verbose_dt: float, band=BETA_BAND) -> np.ndarray:
    """Indices k of rfft bins with band[0] < f_k < band[1] (utils.py:24-26)."""
    freq = np.fft.rfftfreq(W, units2sec(verbose_dt))
    return np.where((freq > band[0]) & (freq < band[1]))[0].astype(np.int32)


def twiddles(W: int, bins) -> tuple[np.ndarray, np.ndarray]:
    """cos/sin(2 pi k n / W) for the selected bins, fp64, shape (n_bins, W).
    The phase is reduced exactly in integers before the float conversion."""
    n = np.arange(W, dtype=np.int64)
    k = np.asarray(bins, dtype=np.int64)[:, None]
    ph = 2.0 * np.pi * ((k * n) % W).astype(np.float64) / W
    return np.ascontiguousarray(np.cos(ph)), np.ascontiguousarray(np.sin(ph))


def butter_bandpass(verbose_dt: float, lowcut=12, highcut=30, order=2):
    """band_pass_envelope(signal, 1/psd_dt, order=2) filter design (utils.py:808-812)."""
    fs = 1 / units2sec(verbose_dt)
    nyq = 0.5 * fs
    b, a = butter(order, [lowcut / nyq, highcut / nyq], btype="band")
    return b, a, lfilter_zi(b, a)
