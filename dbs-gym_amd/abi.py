"""ctypes mirror of include/kura.h and the loader for libkura.so.

The C ABI is the drop-in boundary: Python host code
builds a :class:`KuraConfig`, hands device pointers (``tensor.data_ptr()``) to
``kura_step``/``kura_reset`` and never touches the numerics.  There is no CPU
fallback: if the HIP library is missing, :func:`load_library` raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_int64, c_uint8, c_void_p

KURA_ABI_VERSION = 2   # include/kura.h (2: KuraConfig.coupling, AUTO = BF16X3)
KURA_S_MAX = 32
KURA_MAX_BINS = 32
KURA_NSTATS = 8

# per-env failure bits (kura.h KURA_F_*)
KURA_F_MAX_STEPS = 1
KURA_F_NONFINITE = 2
KURA_F_GRID = 8
KURA_F_BARRIER = 16
KURA_F_BOUNDS = 32     # KURA_DEBUG builds only
FLAG_NAMES = {
    KURA_F_MAX_STEPS: "The maximum number of solver steps was reached",   # diffrax's message (throw=True)
    KURA_F_NONFINITE: "non-finite (NaN/Inf) state or RHS",
    KURA_F_GRID: "save grid outside [2, KURA_S_MAX] samples",
    KURA_F_BARRIER: "split-group barrier timed out",
    KURA_F_BOUNDS: "device access outside its buffer (KURA_DEBUG build)",
}

KURA_REC_NAIVE = 0
KURA_REC_GAUSSIAN = 1
KURA_R_BBPOW = 1
KURA_R_TEMP_CONST = 2
KURA_R_BBPOW_THR = 3

# reward_func names of the reference (environment/env.py:323-330)
REWARD_KINDS = {
    "bbpow_action": KURA_R_BBPOW,
    "temp_const_action": KURA_R_TEMP_CONST,
    "bbpow_threth_action": KURA_R_BBPOW_THR,
}
# coupling arithmetic (kura.h KURA_COUPLING_*): "auto" = bf16x3 at every N
KURA_COUPLING_AUTO = 0
KURA_COUPLING_F32 = 1
KURA_COUPLING_BF16X3 = 2
COUPLINGS = {"auto": KURA_COUPLING_AUTO, "f32": KURA_COUPLING_F32, "bf16x3": KURA_COUPLING_BF16X3}


def coupling_of(cfg) -> str:
    """The arithmetic a config resolves to (kura.h kura_coupling_of)."""
    c = int(cfg.coupling)
    if c == KURA_COUPLING_AUTO:
        c = KURA_COUPLING_BF16X3
    return {KURA_COUPLING_F32: "f32", KURA_COUPLING_BF16X3: "bf16x3"}[c]


# recording_kernel names (environment/env.py:333-338)
REC_KERNELS = {"naive": KURA_REC_NAIVE, "gaussian": KURA_REC_GAUSSIAN}

_ERRORS = {
    -1: ValueError,
    -2: RuntimeError,
    -3: MemoryError,
    -4: NotImplementedError,
    -5: RuntimeError,
}


class KuraConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", c_int32),
        ("n_osc", c_int32),
        ("n_envs", c_int32),
        ("window", c_int32),
        ("n_elec", c_int32),
        ("n_rec", c_int32),
        ("rec_kernel", c_int32),
        ("reward_kind", c_int32),
        ("episode_steps", c_int32),
        ("max_steps", c_int32),
        ("n_bins", c_int32),
        ("bins", c_int32 * KURA_MAX_BINS),
        ("padlen", c_int32),
        ("episode_cap", c_int32),
        ("part_osc", c_int32),
        ("coupling", c_int32),
        ("reserved_i", c_int32 * 1),
        ("dt", c_double),
        ("width", c_double),
        ("pause", c_double),
        ("transient_len", c_double),
        ("act_lo", c_double),
        ("act_hi", c_double),
        ("dbs_lo", c_double),
        ("dbs_hi", c_double),
        ("bw_b", c_double * 5),
        ("bw_a", c_double * 5),
        ("bw_zi", c_double * 4),
        ("reserved_d", c_double * 4),
        ("rtol", c_float),
        ("atol", c_float),
        ("kn", c_float),
        ("dt0", c_float),
        ("reserved_f", c_float * 4),
    ]


# exported by the KURA_DEBUG build (libkura_debug.so) only
_DEBUG_SYMBOLS = {
    "kura_debug_read_workspace": (c_int, [c_void_p, c_void_p, c_int64]),
    "kura_debug_gemm_dump": (c_int, [c_void_p, c_void_p, c_int]),
}

_SYMBOLS = {
    # name: (restype, argtypes)
    "kura_create": (c_int, [POINTER(KuraConfig), c_int, POINTER(c_void_p)]),
    "kura_destroy": (c_int, [c_void_p]),
    "kura_last_error": (ctypes.c_char_p, []),
    "kura_abi_version": (c_int, []),
    "kura_set_coupling": (c_int, [c_void_p, c_void_p]),
    "kura_set_env_params": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "kura_set_spectral": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kura_reset": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "kura_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p]),
    "kura_reward": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "kura_reward_n": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_int,
                              c_void_p, c_void_p, c_void_p]),
    "kura_get_state": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "kura_set_state": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "kura_get_spec": (c_int, [c_void_p, c_void_p]),
    "kura_set_spec": (c_int, [c_void_p, c_void_p]),
    "kura_set_env_gain": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "kura_psd_bbpow": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_double, c_double, c_double, c_void_p,
                               c_void_p]),
    "kura_episode_bbpow": (c_int, [c_void_p, c_void_p, c_double, c_double, c_double, c_void_p, c_void_p]),
    "kura_envelope_stats": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    "kura_episode_envelope_stats": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "kura_get_stats": (c_int, [c_void_p, c_void_p, c_int]),
    "kura_get_env_flags": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kura_set_row_capture": (c_int, [c_void_p, c_void_p]),
    "kura_set_transient_capture": (c_int, [c_void_p, c_void_p]),
    "kura_set_transient_rows": (c_int, [c_void_p, c_void_p]),
    "kura_transient_len": (c_int, [c_void_p]),
    "kura_get_stamps": (c_int, [c_void_p, c_void_p]),
    "kura_selftest_math": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
    "kura_selftest_gemm": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
    "kura_selftest_coupling": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int]),
}

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "csrc", "libkura.so")

_lib = None


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libkura.so (built by ``__graft_entry__.build()``).  Raises if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("KURA_LIB") or LIB_PATH  # KURA_LIB: an alternative build (A/B diagnostics)
    if not os.path.exists(p):
        raise RuntimeError(
            f"libkura.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP library is the only implementation of the step path; there is no CPU fallback)")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in _DEBUG_SYMBOLS.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    if lib.kura_abi_version() != KURA_ABI_VERSION:
        raise RuntimeError("libkura ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


class KuraSolverError(RuntimeError):
    """A solve failed inside kura_step/kura_reset (the reference's diffeqsolve
    raises in these cases, diffrax throw=True, env.py:261-270).  ``envs``:
    failing env indices, ``flags``: their KURA_F_* bits."""

    def __init__(self, what, envs, flags):
        self.envs, self.flags = list(envs), list(flags)
        kinds = sorted({name for f in self.flags for bit, name in FLAG_NAMES.items() if f & bit})
        shown = ", ".join(f"{e}:{f}" for e, f in list(zip(self.envs, self.flags))[:8])
        super().__init__(f"{what}: {'; '.join(kinds)} (env:flags {shown}{' ...' if len(self.envs) > 8 else ''})")


def describe_flags(f: int) -> str:
    return "; ".join(name for bit, name in FLAG_NAMES.items() if f & bit) or "ok"


def check(lib: ctypes.CDLL, rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.kura_last_error()
        msg = msg.decode() if msg else ""
        raise _ERRORS.get(rc, RuntimeError)(f"{what} failed ({rc}): {msg}")


def ptr(a) -> int | None:
    """Raw address of a numpy array or torch tensor (None passes NULL)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


__all__ = [
    "KuraConfig", "load_library", "check", "ptr", "LIB_PATH", "KuraSolverError", "describe_flags",
    "KURA_F_MAX_STEPS", "KURA_F_NONFINITE", "KURA_F_GRID", "KURA_F_BARRIER",
    "KURA_ABI_VERSION", "KURA_S_MAX", "KURA_MAX_BINS", "REWARD_KINDS", "REC_KERNELS",
    "KURA_REC_NAIVE", "KURA_REC_GAUSSIAN", "KURA_R_BBPOW", "KURA_R_TEMP_CONST", "KURA_R_BBPOW_THR",
    "KURA_COUPLING_AUTO", "KURA_COUPLING_F32", "KURA_COUPLING_BF16X3", "COUPLINGS", "coupling_of",
    "c_int64", "c_uint8",
]
