"""ctypes binding of ``libcirculant_fft.so`` (the HIP/gfx950 library).

There is no fallback: if the shared library is missing or fails to load, every
entry point raises.  Build it with ``__graft_entry__.build()`` or
``make -C circulantpreconditioner_amd/csrc``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libcirculant_fft.so")

_lock = threading.Lock()
_lib = None

# error codes (petscerror.h values), include/circulant_fft.h
CFP_SUCCESS = 0


class CirculantError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[cfp error {code}] {msg}")
        self.code = code


def _declare(L) -> None:
    i64, u64, dp, vp, c_int = ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int
    P = ctypes.POINTER
    sig = {
        "cfp_version": ([], ctypes.c_char_p),
        "cfp_last_error": ([], ctypes.c_char_p),
        "cfp_device_count": ([P(c_int)], c_int),
        "cfp_stream_sync": ([vp], c_int),
        "cfp_device_copy": ([vp, vp, ctypes.c_size_t, vp], c_int),
        "cfp_plan_create": ([P(vp), i64, i64, i64, c_int], c_int),
        "cfp_plan_destroy": ([vp], c_int),
        "cfp_plan_set_symbol_transport": ([vp, dp], c_int),
        "cfp_plan_set_symbol_separable": ([vp, dp, dp, dp, dp], c_int),
        "cfp_plan_set_diag": ([vp, dp, c_int], c_int),
        "cfp_plan_get_diag": ([vp, dp, vp], c_int),
        "cfp_plan_symbol_version": ([vp, P(u64)], c_int),
        "cfp_plan_apply": ([vp, dp, dp, vp], c_int),
        "cfp_plan_apply_ex": ([vp, dp, dp, vp, vp], c_int),
        "cfp_plan_apply_with_diag": ([vp, dp, dp, dp, vp], c_int),
        "cfp_plan_apply_host": ([vp, dp, dp], c_int),
        "cfp_plan_apply_with_diag_host": ([vp, dp, dp, dp], c_int),
        "cfp_plan_forward": ([vp, dp, dp, vp], c_int),
        "cfp_plan_backward": ([vp, dp, dp, vp], c_int),
        "cfp_plan_set_chunking": ([vp, i64], c_int),
        "cfp_plan_set_graph": ([vp, c_int], c_int),
        "cfp_plan_set_schedule": ([vp, c_int], c_int),
        "cfp_plan_set_three_pass_shape": ([vp, c_int, c_int], c_int),
        "cfp_rplan_create": ([P(vp), i64, i64, i64, c_int], c_int),
        "cfp_rplan_destroy": ([vp], c_int),
        "cfp_rplan_set_symbol_transport": ([vp, P(ctypes.c_double)], c_int),
        "cfp_rplan_apply": ([vp, vp, vp, vp], c_int),
        "cfp_rplan_num_passes": ([vp, P(c_int)], c_int),
        "cfp_rplan_time_passes": ([vp, vp, vp, c_int, P(ctypes.c_double), vp], c_int),
        "cfp_rplan_set_schedule": ([vp, c_int], c_int),
        "cfp_rplan_schedule": ([vp, P(c_int)], c_int),
        "cfp_plan_num_passes": ([vp, P(c_int)], c_int),
        "cfp_plan_pass_info": ([vp, c_int, P(c_int), P(c_int), P(i64), P(c_int), P(c_int)], c_int),
        "cfp_plan_time_passes": ([vp, dp, dp, c_int, dp, vp], c_int),
        "cfp_plan_profile_begin": ([vp, c_int, c_int], c_int),
        "cfp_plan_profile_end": ([vp, dp, ctypes.POINTER(c_int)], c_int),
        "cfp_pointwise_divide": ([dp, dp, dp, i64, vp], c_int),
        "cfp_scale": ([dp, ctypes.c_double, ctypes.c_double, i64, vp], c_int),
        "cfp_fill_uniform": ([dp, i64, u64, i64, vp], c_int),
        "cfp_build_diag_3d": ([dp, dp, dp, dp, i64, i64, i64, dp, vp], c_int),
        "cfp_transport_symbol_1d": ([i64, dp], c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    # optional groups (declared in include/circulant_fft_dist.h, include/pcshell_fft3d.h)
    from . import _lib_ext
    _lib_ext.declare(L)


def lib():
    """Load the HIP library (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libcirculant_fft.so not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            _declare(L)
            _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != CFP_SUCCESS:
        raise CirculantError(rc, lib().cfp_last_error().decode(errors="replace"))


def exported_symbols() -> list:
    """Names of every cfp_* / PETSc-boundary function the library must export."""
    names = []
    for hdr in ("circulant_fft.h", "circulant_fft_dist.h", "pcshell_fft3d.h", "petsc_mini.h",
                "transport_equation.h", "wave_system.h", "circulant_fft_real.h", "mesh_unstructured.h"):
        path = os.path.join(os.path.dirname(_HERE), "include", hdr)
        if os.path.exists(path):
            names += _parse_decls(path)
    return names


def _parse_decls(path: str) -> list:
    import re
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    out = []
    txt = re.sub(r"^\s*typedef[^;]*;", "", txt, flags=re.M)  # function-pointer typedefs are not exports
    for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w]*\s*\**\s*([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", txt, flags=re.M):
        name = m.group(1)
        if name not in ("if", "while", "return", "sizeof") and len(name) > 2:
            out.append(name)
    return out
