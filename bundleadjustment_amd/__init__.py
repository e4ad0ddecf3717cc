"""bundleadjustment_amd — MI355X-native replacement for the Ceres Problem/Solve
bundle-adjustment path of MatteoWohlrapp/BundleAdjustment.

The numeric work runs in hand-written HIP kernels for gfx950 behind the C-ABI
of include/ba_hip.h (libba_hip.so).  This package is the thin host side:
ctypes binding, problem container, synthetic problem generator, and the
optimizer classes that mirror the reference's API (Optimizer.h:196-289).
"""
from .problem import Problem, make_config, make_synthetic, shard_points, HUBER_A  # noqa: F401
from .solver import Options, Solver, Summary, solve  # noqa: F401

__all__ = ["Problem", "make_config", "make_synthetic", "shard_points", "HUBER_A", "Options", "Solver", "Summary",
           "solve"]
