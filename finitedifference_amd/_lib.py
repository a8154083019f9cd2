"""ctypes binding of libburgers_hip.so (C ABI: include/burgers.h).

The product path has exactly one compute backend: the HIP library built for
gfx950 (finitedifference_amd/csrc, ``python -m finitedifference_amd.build`` or
``__graft_entry__.build()``).  There is no CPU fallback: if the library is
missing, or no MI355X is visible, every compute call raises.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libburgers_hip.so")
ABI_VERSION = 15

BURG_OK, BURG_EINVAL, BURG_ESHAPE, BURG_EHIP, BURG_EHALO = 0, -1, -2, -3, -4
BURG_ENOMEM, BURG_ENOCONV, BURG_ENAN, BURG_ESTATE = -5, -6, -7, -8
SOLVERS = {"march": 0, "newton": 1}
ENGINES = {"stream": 0, "tiles": 1, "pipe": 2}

# Every symbol include/burgers.h declares (checked by tests/test_capi.py).
EXPORTS = (
    "burg_abi_version", "burg_last_error", "burg_ctx_create", "burg_ctx_create_slab",
    "burg_slab_connect", "burg_slab_verify", "burg_slab_halo_note", "burg_slab_halo_mode", "burg_ctx_destroy", "burg_set_problem", "burg_set_options",
    "burg_residual", "burg_slab_residual", "burg_jvp", "burg_block_solve", "burg_run", "burg_upload_state",
    "burg_advance", "burg_download_state", "burg_set_engine", "burg_trajectory",
    "burg_reserve_trajectory", "burg_trajectory_ex", "burg_reserve_trajectory_ex",
    "burg_trajectory_plan", "burg_trajectory_retained", "burg_trajectory_copy",
    "burg_sweep_device", "burg_pod_rsvd_device",
    "burg_kernel_bench", "burg_sweep", "burg_ecsw_matrix", "burg_ecsw_block_device", "burg_lspg",
    "burg_pod", "burg_pod_rsvd", "burg_run_npy", "burg_run_npy_ex", "burg_build_id",
    "burg_build_flags", "burg_ring_audit", "burg_ring_audit_ex",
)
KERNELS = {"residual": 0, "jvp": 1}


class BurgStats(ctypes.Structure):
    """Mirror of struct burg_stats (include/burgers.h)."""
    _fields_ = [
        ("steps", ctypes.c_int64),
        ("tile_marches", ctypes.c_int64),
        ("passes", ctypes.c_int64),
        ("max_passes", ctypes.c_int32),
        ("unconverged_steps", ctypes.c_int32),
        ("newton_updates", ctypes.c_int64),
        ("newton_max_updates", ctypes.c_int32),
        ("par_passes", ctypes.c_int32),
        ("loop_ms", ctypes.c_double),
        ("flush_ms", ctypes.c_double),
        ("march_kernel_ms", ctypes.c_double),
        ("march_launches", ctypes.c_int64),
        ("last_rel", ctypes.c_double),
        ("tail_passes", ctypes.c_int64),
        ("engine", ctypes.c_int32),
        ("stream_w", ctypes.c_int32),
        ("stream_tiles", ctypes.c_int64),
        ("stall_spins", ctypes.c_int64),
        ("slow_diagonals", ctypes.c_int64),
        ("stream_launches", ctypes.c_int64),
        ("slow_ticks", ctypes.c_int64),
        ("ieee_diagonals", ctypes.c_int64),
        ("comm_polls", ctypes.c_int64),
        ("nonfinite_diagonals", ctypes.c_int64),
        ("paired_launches", ctypes.c_int64),
        ("ramp_ms", ctypes.c_double),
        ("halo_wait_ms", ctypes.c_double),
        ("south_waits_local", ctypes.c_int64),
        ("south_waits_halo", ctypes.c_int64),
        ("south_wait_ms_local", ctypes.c_double),
        ("south_wait_ms_halo", ctypes.c_double),
        ("bounds_checks", ctypes.c_int64),
        ("bounds_hits", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class BurgersError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libburgers_hip error {code}: {msg}")
        self.code = code


class NotConvergedWarning(UserWarning):
    pass


_lib = None
_lock = threading.Lock()
_D = ctypes.POINTER(ctypes.c_double)
_I32 = ctypes.POINTER(ctypes.c_int32)
_VP = ctypes.c_void_p


def load(path=None):
    """Load (once) and return the HIP library; raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("BURG_LIB") or LIB_PATH  # BURG_LIB: A/B builds
        if not os.path.exists(p):
            raise RuntimeError(
                f"{p} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()' or make -C "
                "finitedifference_amd/csrc). There is no CPU fallback.")
        # One HIP runtime per process: torch ships its own libamdhip64 under
        # the same soname.  Loaded first, it is the runtime this library binds
        # to; loaded after a HIP runtime is up, torch finds no GPU.  The
        # decoder-ECSW variants (ecsw.py) and the benches use both.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(p)
        sig = {
            "burg_abi_version": (ctypes.c_int, []),
            "burg_last_error": (ctypes.c_char_p, []),
            "burg_build_id": (ctypes.c_char_p, []),
            "burg_ring_audit": (ctypes.c_int, [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_int64)]),
            "burg_ring_audit_ex": (ctypes.c_int, [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_int64)]),
            "burg_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(_VP)]),
            "burg_ctx_create_slab": (ctypes.c_int, [ctypes.c_int] * 7 + [ctypes.c_char_p,
                                                                         ctypes.POINTER(_VP)]),
            "burg_slab_connect": (ctypes.c_int, [_VP]),
            "burg_slab_verify": (ctypes.c_int, [_VP]),
            "burg_slab_halo_note": (ctypes.c_char_p, [_VP]),
            "burg_slab_halo_mode": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_int)]),
            "burg_ctx_destroy": (None, [_VP]),
            "burg_set_problem": (ctypes.c_int, [_VP, _D, _D, _D, _D, ctypes.c_double]),
            "burg_set_options": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_double, ctypes.c_int]),
            "burg_residual": (ctypes.c_int, [_VP, _D, _D, _D, _D]),
            "burg_slab_residual": (ctypes.c_int, [_VP, _D, _D, _D, _D, _D, _D]),
            "burg_jvp": (ctypes.c_int, [_VP, _D, _D, _D]),
            "burg_block_solve": (ctypes.c_int, [_VP, _D, _D, _D]),
            "burg_run": (ctypes.c_int, [_VP, _D, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_double, _D, ctypes.c_int64, ctypes.c_int,
                                        ctypes.POINTER(BurgStats), _I32, _D]),
            "burg_upload_state": (ctypes.c_int, [_VP, _D]),
            "burg_advance": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(BurgStats)]),
            "burg_download_state": (ctypes.c_int, [_VP, _D]),
            "burg_trajectory": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(BurgStats)]),
            "burg_reserve_trajectory": (ctypes.c_int, [_VP, ctypes.c_int]),
            "burg_trajectory_ex": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.POINTER(BurgStats)]),
            "burg_reserve_trajectory_ex": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int]),
            "burg_trajectory_plan": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int,
                                                     ctypes.POINTER(ctypes.c_int),
                                                     ctypes.POINTER(ctypes.c_int64),
                                                     ctypes.POINTER(ctypes.c_int64)]),
            "burg_trajectory_retained": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int64),
                                                         ctypes.POINTER(ctypes.c_int64),
                                                         ctypes.POINTER(ctypes.c_int)]),
            "burg_trajectory_copy": (ctypes.c_int, [_VP, ctypes.c_int64, ctypes.c_int64,
                                                     ctypes.c_void_p, ctypes.c_int64,
                                                     ctypes.c_int]),
            "burg_set_engine": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
            "burg_kernel_bench": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _D]),
            "burg_ecsw_matrix": (ctypes.c_int, [_VP, ctypes.c_int, _D, _D, ctypes.c_int, _D, _D,
                                                ctypes.POINTER(BurgStats)]),
            "burg_ecsw_block_device": (ctypes.c_int, [_VP, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_int, ctypes.c_void_p,
                                                      ctypes.c_void_p,
                                                      ctypes.POINTER(ctypes.c_float)]),
            "burg_lspg": (ctypes.c_int, [_VP, _D, ctypes.c_int, ctypes.c_int, _D, ctypes.c_int,
                                         ctypes.c_double, ctypes.c_double, _D, ctypes.c_int64,
                                         _D, ctypes.c_int64, _I32, _D, _D,
                                         ctypes.POINTER(BurgStats)]),
            "burg_pod": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.c_int, _D,
                                        ctypes.c_int, _D, _D, _D]),
            "burg_pod_rsvd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.c_int, _D,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, _D, _D, _D,
                                             _D]),
            "burg_run_npy": (ctypes.c_int, [_VP, _D, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                            ctypes.POINTER(BurgStats)]),
            "burg_run_npy_ex": (ctypes.c_int, [_VP, _D, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_char_p, ctypes.c_int,
                                               ctypes.POINTER(BurgStats)]),
            "burg_build_flags": (ctypes.c_char_p, []),
            "burg_sweep": (ctypes.c_int, [_VP, ctypes.c_int, _D, _D, ctypes.c_int,
                                          ctypes.POINTER(_D), ctypes.c_int64, ctypes.c_int,
                                          ctypes.POINTER(BurgStats)]),
            "burg_sweep_device": (ctypes.c_int, [_VP, ctypes.c_int, _D, _D, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                                 ctypes.POINTER(BurgStats)]),
            "burg_pod_rsvd_device": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int, _D, _D, _D, _D]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.burg_abi_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"{p}: ABI version {v}, expected {ABI_VERSION}")
        _lib = lib
        return lib


_CSRC = os.path.join(_HERE, "csrc")


def source_id(csrc=_CSRC):
    """The digest burg_build_id() reports, computed from the sources in this
    checkout (csrc/*.h and *.hip in byte order, then csrc/Makefile and
    include/burgers.h -- the Makefile's BUILD_ID_SRCS)."""
    import glob
    import hashlib
    names = sorted(os.path.basename(f) for f in glob.glob(os.path.join(csrc, "*.hip")) +
                   glob.glob(os.path.join(csrc, "*.h")))
    files = [os.path.join(csrc, n) for n in names]
    files += [os.path.join(csrc, "Makefile"),
              os.path.join(os.path.dirname(_HERE), "include", "burgers.h")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id():
    """burg_build_id() of the loaded library."""
    return load().burg_build_id().decode()


def build_flags():
    """burg_build_flags() of the loaded library: 'HIPFLAGS | knobs: ...'
    ('knobs: none' for the default build; A/B and race-screen variants name
    their -D knobs, csrc/Makefile VARIANT / KNOBS)."""
    return load().burg_build_flags().decode()


def is_default_build():
    return build_flags().endswith("knobs: none")


def ring_audit(W, num_steps, snap_every=1, ring_cap=0, paired=False, paired_layout=False):
    """burg_ring_audit_ex as a dict (host-only; no GPU needed); paired: the
    paired-halves W = 16 kernel's walk; paired_layout (with paired): its store
    wave's paired sweep layout (BURG_AUDIT_PAIRED_LAYOUT)."""
    rep = (ctypes.c_int64 * 9)()
    flags = (1 if paired else 0) | (2 if paired_layout else 0)
    check(load().burg_ring_audit_ex(int(W), int(num_steps), int(snap_every), int(ring_cap),
                                    flags, rep))
    keys = ("accesses", "max_entry", "entries_per_tile", "out_of_range", "walk_mismatch",
            "retained_overwritten", "early_overwrite", "retained_states", "snap_every")
    return dict(zip(keys, list(rep)))


def check(code, allow=()):
    if code == BURG_OK or code in allow:
        return code
    msg = load().burg_last_error().decode(errors="replace")
    raise BurgersError(code, msg)


def dptr(a):
    """double* of a C-contiguous float64 array (None -> NULL)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous, "need C-contiguous float64"
    return a.ctypes.data_as(_D)


def iptr(a):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_I32)
