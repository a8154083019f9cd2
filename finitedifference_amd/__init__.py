"""finitedifference_amd -- MI355X-native FOM hot path of SADPR/FiniteDifference.

The 2D inviscid Burgers implicit time loop (reference hypernet2D.py /
run_fom.py) on hand-written HIP kernels for gfx950, behind the reference's
own Python API (hypernet2D.py here).  See DESIGN.md.
"""
from .grid import fom_coefficients, make_2D_grid
from .hypernet2D import (JacobianOperator, compute_error, get_ops, get_saved_params,
                         inviscid_burgers_exact_jac2D, inviscid_burgers_implicit2D,
                         inviscid_burgers_res2D_alt, load_or_compute_snaps, make_ddx,
                         newton_raphson, param_to_snap_fn)
from .solver import FOMContext, get_context

__all__ = [
    "make_2D_grid", "fom_coefficients", "make_ddx", "get_ops", "inviscid_burgers_implicit2D",
    "inviscid_burgers_res2D_alt", "inviscid_burgers_exact_jac2D", "JacobianOperator",
    "newton_raphson", "compute_error", "param_to_snap_fn", "get_saved_params",
    "load_or_compute_snaps", "FOMContext", "get_context",
]
