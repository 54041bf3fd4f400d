"""Per-env MT19937 streams for the host draws of reset(), in native code
(``csrc/kura_hostrng.c`` -> ``libkura_host.so``).

The reference draws from NumPy's legacy RandomState (env.py:291, :595-598;
utils.py:819-823, :868, :927).  ``StreamBank`` holds the states of B such
streams in one array and draws for many envs per call; ``Stream`` is one env's
view with the RandomState methods the host code uses.  Every draw is bit for
bit what ``numpy.random.RandomState(seed)`` returns for the same calls
(tests/test_hostrng.py); methods it does not implement natively (``shuffle``,
``choice`` with a size or p, ...) run on a scratch RandomState loaded with this stream's state
and store the advanced state back, so any RandomState call is available with
the same results.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "libkura_host.so")
_lib = None

# kh_mt (kura_hostrng.c): the fields of RandomState.get_state()
STATE_DTYPE = np.dtype([("key", "<u4", (624,)), ("pos", "<i4"), ("has_gauss", "<i4"), ("gauss", "<f8")], align=True)


def lib():
    """libkura_host.so (built by __graft_entry__.build(); raises if absent)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise ImportError(f"{_LIB_PATH} is missing: run __graft_entry__.build()")
        L = ctypes.CDLL(_LIB_PATH)
        P, I64, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
        L.kh_state_size.restype = ctypes.c_int
        L.kh_state_size.argtypes = []
        L.kh_randint.restype = I64
        L.kh_randint.argtypes = [P, I64, I64, I64]
        for name, args in (("kh_seed", [P, P, P, I64]),
                           ("kh_random_sample", [P, P, I64, I64, P]),
                           ("kh_uniform", [P, P, I64, P, P, I64, P]),
                           ("kh_normal", [P, P, I64, P, P, I64, P]),
                           ("kh_randn", [P, I64, I64, P]),
                           ("kh_remove_nonpositive", [P, P, I64, P, I64]),
                           ("kh_perturbations", [P, P, I64, P, I64, I64, D, P, P]),
                           ("kh_interp", [P, I64, P, P, I64, D, D, P])):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = args
        if L.kh_state_size() != STATE_DTYPE.itemsize:
            raise ImportError("libkura_host.so: kh_mt layout differs from hostrng.STATE_DTYPE")
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _rows(rows) -> np.ndarray:
    r = np.ascontiguousarray(rows, dtype=np.int64)
    if r.ndim != 1:
        raise ValueError("rows must be 1-D")
    if len(r) > 1 and len(np.unique(r)) != len(r):
        raise ValueError("rows must be distinct (the streams are drawn in parallel)")
    return r


def _seed_u32(seed) -> int:
    """RandomState's integer seed range (0 <= seed < 2**32)."""
    s = int(seed)
    if s != seed or not 0 <= s <= 0xFFFFFFFF:
        raise ValueError(f"seed {seed!r}: an integer in [0, 2**32) is required")
    return s


class StreamBank:
    """B MT19937 streams, stream b seeded as ``RandomState(seeds[b])``."""

    def __init__(self, seeds):
        seeds = [_seed_u32(s) for s in seeds]
        self.state = np.zeros(len(seeds), dtype=STATE_DTYPE)
        self.seed(np.arange(len(seeds)), seeds)

    def __len__(self):
        return len(self.state)

    def seed(self, rows, seeds):
        rows = _rows(rows)
        sd = np.asarray([_seed_u32(s) for s in np.atleast_1d(seeds)], dtype=np.uint32)
        if len(sd) != len(rows):
            raise ValueError("seed: one seed per row")
        lib().kh_seed(_ptr(self.state), _ptr(rows), _ptr(sd), len(rows))

    def random_sample(self, rows, m: int) -> np.ndarray:
        rows = _rows(rows)
        out = np.empty((len(rows), int(m)))
        lib().kh_random_sample(_ptr(self.state), _ptr(rows), len(rows), int(m), _ptr(out))
        return out

    def uniform(self, rows, low, high, m: int) -> np.ndarray:
        rows = _rows(rows)
        lo = np.ascontiguousarray(np.broadcast_to(np.asarray(low, np.float64), (len(rows),)))
        hi = np.ascontiguousarray(np.broadcast_to(np.asarray(high, np.float64), (len(rows),)))
        if not np.all(np.isfinite(hi - lo)):
            raise OverflowError("Range exceeds valid bounds")
        out = np.empty((len(rows), int(m)))
        lib().kh_uniform(_ptr(self.state), _ptr(rows), len(rows), _ptr(lo), _ptr(hi), int(m), _ptr(out))
        return out

    def normal(self, rows, loc, scale, m: int) -> np.ndarray:
        rows = _rows(rows)
        mu = np.ascontiguousarray(np.broadcast_to(np.asarray(loc, np.float64), (len(rows),)))
        sd = np.ascontiguousarray(np.broadcast_to(np.asarray(scale, np.float64), (len(rows),)))
        if len(rows) and np.min(sd) < 0:
            raise ValueError("scale < 0")
        out = np.empty((len(rows), int(m)))
        lib().kh_normal(_ptr(self.state), _ptr(rows), len(rows), _ptr(mu), _ptr(sd), int(m), _ptr(out))
        return out

    def remove_nonpositive(self, rows, x: np.ndarray) -> None:
        """model_setup.remove_negative_w0 (utils.py:819-823) on each row of the
        C-contiguous float64 (len(rows), m) array x, in place, row i drawing
        from stream rows[i]."""
        rows = _rows(rows)
        if x.dtype != np.float64 or not x.flags.c_contiguous or x.ndim != 2 or x.shape[0] != len(rows):
            raise ValueError("remove_nonpositive: x must be C-contiguous float64 of shape (len(rows), m)")
        lib().kh_remove_nonpositive(_ptr(self.state), _ptr(rows), len(rows), _ptr(x), x.shape[1])

    def perturbations(self, rows, initial: np.ndarray, M: int, step_scale: float) -> np.ndarray:
        """model_setup.generate_perturbations (env.py:21-57) for each row of
        initial (len(rows), m), row i drawing from stream rows[i]:
        (len(rows), M + 1, m) float64."""
        rows = _rows(rows)
        x = np.ascontiguousarray(initial, dtype=np.float64)
        if x.ndim != 2 or x.shape[0] != len(rows) or x.shape[1] < 2:
            raise ValueError("perturbations: initial must be (len(rows), m >= 2)")
        out = np.empty((len(rows), int(M) + 1, x.shape[1]))
        tmp = np.empty_like(x)
        lib().kh_perturbations(_ptr(self.state), _ptr(rows), len(rows), _ptr(x), x.shape[1], int(M),
                               float(step_scale), _ptr(out), _ptr(tmp))
        return out

    def randint(self, row: int, low: int, high: int) -> int:
        """RandomState.randint(low, high) (size=None) on stream row."""
        return int(lib().kh_randint(_ptr(self.state), int(row), int(low), int(high)))

    def randn(self, row: int, m: int) -> np.ndarray:
        out = np.empty(int(m))
        lib().kh_randn(_ptr(self.state), int(row), int(m), _ptr(out))
        return out

    def get_state(self, row: int):
        r = self.state[row]
        return ("MT19937", r["key"].copy(), int(r["pos"]), int(r["has_gauss"]), float(r["gauss"]))

    def set_state(self, row: int, st):
        name, key, pos, has_gauss, gauss = st[:5] if len(st) >= 5 else (*st, 0, 0.0)
        if name != "MT19937":
            raise ValueError(f"set_state: {name!r} is not an MT19937 state")
        key = np.asarray(key, dtype=np.uint32)
        if key.shape != (624,):
            raise ValueError("set_state: the MT19937 key must have 624 words")
        r = self.state[row:row + 1]
        r["key"][0] = key
        r["pos"] = int(pos)
        r["has_gauss"] = int(has_gauss)
        r["gauss"] = float(gauss)

    def stream(self, row: int) -> "Stream":
        return Stream(self, row)


_SCRATCH = None


def _scratch() -> np.random.RandomState:
    global _SCRATCH
    if _SCRATCH is None:
        _SCRATCH = np.random.RandomState(0)
    return _SCRATCH


def _size_len(size) -> int | None:
    if size is None:
        return None
    return int(np.prod(size))


class Stream:
    """One env's stream: the RandomState interface the host code uses."""

    __slots__ = ("bank", "row")

    def __init__(self, bank: StreamBank, row: int):
        self.bank, self.row = bank, int(row)

    def seed(self, seed):
        self.bank.seed([self.row], [seed])

    def get_state(self):
        return self.bank.get_state(self.row)

    def set_state(self, st):
        self.bank.set_state(self.row, st)

    def _shape(self, a: np.ndarray, size):
        if size is None:
            return a[0]
        return a.reshape(size)

    def rand(self, *shape):
        if not shape:
            return self.bank.random_sample([self.row], 1)[0, 0]
        return self.bank.random_sample([self.row], int(np.prod(shape)))[0].reshape(shape)

    def random_sample(self, size=None):
        n = _size_len(size)
        return self._shape(self.bank.random_sample([self.row], 1 if n is None else n)[0], size)

    def uniform(self, low=0.0, high=1.0, size=None):
        if np.ndim(low) or np.ndim(high):
            return self._numpy("uniform", low, high, size)
        n = _size_len(size)
        return self._shape(self.bank.uniform([self.row], low, high, 1 if n is None else n)[0], size)

    def normal(self, loc=0.0, scale=1.0, size=None):
        if np.ndim(loc) or np.ndim(scale):
            return self._numpy("normal", loc, scale, size)
        n = _size_len(size)
        return self._shape(self.bank.normal([self.row], loc, scale, 1 if n is None else n)[0], size)

    def randint(self, low, high=None, size=None, dtype=int):
        if high is None:
            low, high = 0, low
        if size is None and dtype is int and np.ndim(low) == 0 and np.ndim(high) == 0 \
                and 1 <= int(high) - int(low) <= 1 << 32:
            return self.bank.randint(self.row, int(low), int(high))
        return self._numpy("randint", low, high, size, dtype)

    def choice(self, a, size=None, replace=True, p=None):
        """RandomState.choice: one uniform index (size=None, replace, no p) is
        randint(0, len(a)) -- native; anything else runs on the scratch state."""
        if size is None and replace and p is None:
            arr = np.asarray(a)
            pop = int(arr) if arr.ndim == 0 else arr.shape[0]
            if arr.ndim <= 1 and 1 <= pop <= 1 << 32:
                idx = self.bank.randint(self.row, 0, pop)
                return idx if arr.ndim == 0 else arr[idx]
        return self._numpy("choice", a, size, replace, p)

    def randn(self, *shape):
        if not shape:
            return self.bank.randn(self.row, 1)[0]
        return self.bank.randn(self.row, int(np.prod(shape))).reshape(shape)

    def _numpy(self, name, *a, **k):
        rs = _scratch()
        rs.set_state(self.get_state())
        out = getattr(rs, name)(*a, **k)
        self.set_state(rs.get_state())
        return out

    def __getattr__(self, name):
        if name.startswith("_") or not callable(getattr(np.random.RandomState, name, None)):
            raise AttributeError(name)
        return lambda *a, **k: self._numpy(name, *a, **k)


def interp(x: np.ndarray, xp: np.ndarray, fp: np.ndarray, left: float, right: float) -> np.ndarray:
    """numpy.interp(x, xp, fp, left, right) for sorted xp, OpenMP-parallel."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    xp = np.ascontiguousarray(xp, dtype=np.float64)
    fp = np.ascontiguousarray(fp, dtype=np.float64)
    if xp.ndim != 1 or xp.shape != fp.shape or len(xp) < 2:
        raise ValueError("interp: xp and fp must be 1-D of the same length >= 2")
    out = np.empty_like(x)
    lib().kh_interp(_ptr(x), x.size, _ptr(xp), _ptr(fp), len(xp), float(left), float(right), _ptr(out))
    return out
