"""f110qp — MI355X batched MPC/QP solver for the f110-mpc control tick.

Python surface over the C ABI of include/f110qp.h (libf110qp.so, HIP for gfx950):
  capi      ctypes binding (Solver, find_half_spaces[_dev], status codes)
  workload  synthetic tick batches in the ABI layouts
The C++ host mirror of the reference classes (MPC, Constraints, Cost, Model, State, Input)
lives in ../host/.
"""
from . import capi, workload  # noqa: F401
from .capi import Solver, default_config, F110QPError  # noqa: F401

__all__ = ["capi", "workload", "Solver", "default_config", "F110QPError"]
