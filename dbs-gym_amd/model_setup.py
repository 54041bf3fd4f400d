"""Host-side model setup: grid, distances, coupling, conductances, natural
frequencies, locus, RNG-driven reset draws.

These run once per configuration (or once per reset for drift events) on the
host in float64 NumPy, exactly as the reference computes them, and their
results are uploaded through the C ABI.  Each function cites the reference
code it restates.  Random draws use a per-environment legacy
``numpy.random.RandomState`` so that env ``b`` of a batch reproduces the
draw order of a stand-alone reference ``SpatialKuramoto`` seeded the same
way (the reference uses the process-global MT19937, env.py:291,595).
"""
from __future__ import annotations

import numpy as np
from scipy.integrate import quad
from scipy.interpolate import interp1d

from . import hostrng


def neuron_grid_3d(gx: int, gy: int, gz: int, n: int, coord_modif: float = 0.1):
    """utils.py:478-497 generate_neuron_grid_3D (no shuffle).

    ``meshgrid(x, y, z).T.reshape(-1, 3)`` enumerates z slowest, then x, then y,
    i.e. flat index = (z*gx + x)*gy + y (8x + y + 64z on the 8^3 grid).
    """
    if n > gx * gy * gz:
        raise ValueError("Number of neurons should be less than grid size.")
    zz, xx, yy = np.meshgrid(np.arange(gz), np.arange(gx), np.arange(gy), indexing="ij")
    grid = np.stack([xx.ravel(), yy.ravel(), zz.ravel()], axis=1)[:n]
    return grid * coord_modif, grid


def distance_matrix(coords: np.ndarray) -> np.ndarray:
    """utils.py:457-466 create_distance_matrix, vectorised.

    The reference fills the upper triangle with ``np.linalg.norm(c_i - c_j)``
    (a 3-term BLAS dot, then sqrt) and mirrors it.  Here the squares are summed
    as ((x^2 + y^2) + z^2); the BLAS dot of this container fuses the adds, so
    entries can differ by 1 ulp of float64 -- the float32 coupling uploaded to
    the device (jnp.array(alpha) with x64 off) is identical
    (tests/test_golden_reference.py).
    """
    c = np.asarray(coords, dtype=np.float64)
    d = c[:, None, :] - c[None, :, :]
    sq = d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]
    sq = sq + d[..., 2] * d[..., 2]
    D = np.sqrt(sq)
    iu = np.triu_indices(c.shape[0], 1)
    D[iu[1], iu[0]] = D[iu]  # mirror upper triangle exactly like the loop
    np.fill_diagonal(D, 0.0)
    return D


def wavelet_kernel_matrix(distances, amplitude, steepness):
    """utils.py:469-475 (Mexican-hat spatial kernel option)."""
    return (amplitude * (-steepness) * (12 * steepness ** 4 * distances ** 2 - 8 * steepness ** 2)
            * np.exp(-steepness * distances ** 2) / (2 * np.pi))


def coupling_alpha(coords, spatial_kernel="cos", wavelet_amp=1.0, wavelet_steepness=1.0) -> np.ndarray:
    """env.py:219-229: alpha = cos(D) or the wavelet kernel; float64."""
    D = distance_matrix(coords)
    if spatial_kernel == "cos":
        return np.cos(D)
    if spatial_kernel == "wavelet":
        return wavelet_kernel_matrix(D, wavelet_amp, wavelet_steepness)
    raise ValueError(f"Wrong distance matrix type: {spatial_kernel}")


def flat_index(coord, grid_size) -> int:
    """env.py:94,97 (and utils.py:887): c0*gs[2]**2 + c1*gs[1] + c2.

    Kept verbatim for parity although it does not match the grid enumeration
    (electrode [4,3,4] lands on grid point (3,4,4))."""
    return int(coord[0] * grid_size[2] ** 2 + coord[1] * grid_size[1] + coord[2])


def conductance_row(neur_grid, grid_size, coord, conduct_modifier, naive=False) -> np.ndarray:
    """SimpleDBS conductance for one contact, env.py:106-120 / :142-156:
    g = max(0, 1 - dist(grid*conduct_modifier)[idx]); ones if naive."""
    pos = np.asarray(neur_grid, dtype=np.float64) * conduct_modifier
    idx = flat_index(coord, grid_size)
    v = pos - pos[idx]
    sq = v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]
    sq = sq + v[:, 2] * v[:, 2]
    d = np.sqrt(sq)
    d[idx] = 0.0
    if naive:
        return np.ones_like(d)
    g = 1 - d
    return np.where(g < 0.0, 0, g)


def conductances(neur_grid, grid_size, coords_list, conduct_modifier, naive=False) -> np.ndarray:
    return np.stack([conductance_row(neur_grid, grid_size, c, conduct_modifier, naive) for c in coords_list])


# ---- natural frequencies (utils.py:847-942) --------------------------------
_W0_X = [0, 1.8, 2.5, 3.3, 4.5, 5.5, 8, 12.5, 18, 20, 22, 25, 30, 35, 40, 45, 50, 55, 60]


def _w0_inverse_cdf(lf_peak=6, beta_peak=10):
    """Inverse CDF of the degree-10 polynomial spectral prior, utils.py:847-867."""
    y = [6, 7.7, lf_peak, 7.7, 4, 3.5, 4, 5, 5.7, beta_peak, 5.7, 4.9, 2.3, 1.2, 0.8, 0.75, 0.7, 0.7, 0.68]
    x = _W0_X
    poly = np.poly1d(np.polyfit(x, y, 10))
    x_range = np.linspace(np.min(x), 30, 1000)

    def pdf(t):
        return np.maximum(poly(t), 0)

    const, _ = quad(pdf, np.min(x), np.max(x))
    cdf = np.cumsum(pdf(x_range) / const)
    cdf /= cdf[-1]
    return interp1d(cdf, x_range, bounds_error=False, fill_value=(x_range[0], x_range[-1]))


_INV_CDF = None


def w0_from_uniform(u: np.ndarray) -> np.ndarray:
    """The inverse-CDF transform of generate_w0_samples (utils.py:868-882) on
    uniform draws of any shape (elementwise)."""
    global _INV_CDF
    if _INV_CDF is None:
        _INV_CDF = _w0_inverse_cdf()
    f = _INV_CDF
    u = np.asarray(u, dtype=np.float64)
    if u.size < 4096:
        return f(u)
    # interp1d's linear path is numpy.interp on its sorted table with the fill
    # values outside it; hostrng.interp is the same arithmetic, multithreaded
    # (tests/test_hostrng.py checks it against f on the same draws)
    return hostrng.interp(u, f.x, f.y, f.fill_value[0], f.fill_value[1]).reshape(u.shape)


def sample_w0(rs: np.random.RandomState, n: int) -> np.ndarray:
    """utils.py:847-882 generate_w0_samples: inverse-CDF samples (Hz-like)."""
    return w0_from_uniform(rs.rand(n))


def locus_mask(neur_grid, grid_size, locus_coord, locus_size) -> np.ndarray:
    """utils.py:885-891 create_oscillation_locus: 1 inside the unit ball of
    grid*locus_size around the (reference-indexed) locus centre."""
    pos = np.asarray(neur_grid, dtype=np.float64) * locus_size
    idx = flat_index(locus_coord, grid_size)
    v = pos - pos[idx]
    sq = v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]
    sq = sq + v[:, 2] * v[:, 2]
    d = np.sqrt(sq)
    d[idx] = 0.0
    return np.where(1 - d < 0.0, 0., 1.)


def apply_locus_mask(w0, w_locus, lmask):
    """utils.py:902-906."""
    inv = lmask * -1 + 1
    return w0 * inv + w_locus * lmask


def generate_w0_with_locus(rs, n_neurons, grid_size, coord_modif, locus_center, locus_size, wmuL, wsdL):
    """utils.py:909-942: returns (w0_rad, coords, grid, w0_wo_locus_rad, w_locus_rad, mask)."""
    w0_deg = sample_w0(rs, n_neurons)
    coords, grid = neuron_grid_3d(*grid_size, n_neurons, coord_modif=coord_modif)
    lm = locus_mask(grid, grid_size, locus_center, locus_size)
    wl = rs.uniform(low=wmuL - wsdL, high=wmuL + wsdL, size=n_neurons)
    w = apply_locus_mask(w0_deg, wl, lm)
    return w * 0.065, coords, grid, w0_deg * 0.065, wl * 0.065, lm


def remove_negative_w0(rs: np.random.RandomState, w0: np.ndarray) -> np.ndarray:
    """utils.py:819-823 (mutates and returns w0; draws only if needed)."""
    idx = np.where(w0 <= 0.)[0]
    noise = rs.randn(len(idx)) * 0.05
    w0[idx] = np.abs(noise) + np.mean(w0)
    return w0


def initial_phases(rs: np.random.RandomState, n: int, mean=np.pi, sd=0.6) -> np.ndarray:
    """env.py:594-598: theta0 ~ N(mean, sd) with non-positive entries replaced."""
    th = rs.normal(loc=mean, scale=sd, size=n)
    return remove_negative_w0(rs, th)


def generate_perturbations(rs: np.random.RandomState, initial, M=10, step_scale=0.1):
    """env.py:21-57: random walk of the natural frequencies (env2 plasticity)."""
    out = [initial.copy()]
    scale = np.std(initial.copy(), ddof=1)
    for _ in range(M):
        cur = out[-1]
        step = step_scale * scale * rs.randn(len(cur))
        out.append(cur + step)
    return np.array(out)


def directed_stim_masks(grid_points, center, center_idx):
    """utils.py:30-57: three 120-degree azimuthal sectors around the contact."""
    x = grid_points[:, 0] - center[0]
    y = grid_points[:, 1] - center[1]
    theta = np.arctan2(y, x)
    m1 = (theta >= -np.pi / 3) & (theta < np.pi / 3)
    m2 = (theta >= np.pi / 3) & (theta <= np.pi)
    m3 = (theta >= -np.pi) & (theta < -np.pi / 3)
    for m in (m1, m2, m3):
        m[center_idx] = True
    return m1, m2, m3


def directed_conductances(neur_grid, grid_size, elec_coords, g_stim) -> np.ndarray:
    """SimpleDBS directional stimulation (env.py:125-140): every contact's
    conductance times the first 120-degree sector around that contact.  As in
    the reference, the sector's forced-on centre is the LAST contact's index
    (the loop variable elec_idx left over from env.py:93-95) for every contact."""
    last_idx = flat_index(elec_coords[-1], grid_size)
    masks = [directed_stim_masks(neur_grid, np.asarray(c), last_idx)[0] for c in elec_coords]
    return np.asarray(g_stim) * np.stack(masks)
