"""dbs-gym_amd: MI355X-native batched Kuramoto environment (drop-in for
SpatialKuramoto.step()/reset() of NevVerVer/DBS-Gym, environment/env.py).

Import with ``importlib.import_module("dbs-gym_amd")`` (the directory name is
not a Python identifier).  Numerics live in csrc/libkura.so (HIP, gfx950).
"""
from . import abi, configs, model_setup, spectral  # noqa: F401
from .abi import coupling_of, load_library  # noqa: F401
from .configs import reference_params, synthetic_params  # noqa: F401
from .batch import EnvHost, build_batch, fill_driver_arrays, fill_driver_arrays_batch, reset_arrays, reset_draws_batch  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # torch-dependent pieces are imported lazily so host-only helpers stay cheap
    if name in ("KuraSim", "make_config", "auto_part_osc"):
        from . import sim
        return getattr(sim, name)
    if name == "KuraSB3VecEnv":
        from . import sb3
        return sb3.KuraSB3VecEnv
    if name in ("KuraVectorEnv", "SpatialKuramoto"):
        from . import vec_env
        return getattr(vec_env, name)
    raise AttributeError(name)
