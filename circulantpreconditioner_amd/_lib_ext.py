"""ctypes signatures of the slab-distributed plan (include/circulant_fft_dist.h) and of
the PETSc PCSHELL boundary (include/pcshell_fft3d.h, include/petsc_mini.h)."""
from __future__ import annotations

import ctypes


def declare(L) -> None:
    i64, dp, vp, c_int, dbl = ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    P = ctypes.POINTER
    sig = {
        # slab-distributed plan over RCCL
        "cfp_dist_get_unique_id": ([ctypes.c_char_p], c_int),
        "cfp_dist_unique_id_bytes": ([], c_int),
        "cfp_slab_layout": ([i64, i64, i64, c_int, c_int, P(i64)], c_int),
        "cfp_dist_plan_create": ([P(vp), i64, i64, i64, c_int, c_int, ctypes.c_char_p, c_int], c_int),
        "cfp_dist_plan_destroy": ([vp], c_int),
        "cfp_dist_plan_set_symbol_transport": ([vp, dp], c_int),
        "cfp_dist_plan_apply": ([vp, dp, dp, vp], c_int),
        "cfp_dist_plan_local_size": ([vp, P(i64)], c_int),
        "cfp_dist_plan_time_phases": ([vp, dp, dp, c_int, dp, vp], c_int),
        "cfp_dist_plan_num_phases": ([vp, P(c_int)], c_int),
        # mini-PETSc objects + the reference-named callbacks
        "VecCreateSeqHIPWithArray": ([vp, c_int, i64, dp, P(vp)], c_int),
        "VecCreateSeqHIP": ([vp, i64, P(vp)], c_int),
        "VecCreateSeq": ([vp, i64, P(vp)], c_int),
        "VecDestroy": ([P(vp)], c_int),
        "VecGetSize": ([vp, P(i64)], c_int),
        "VecSetValuesHost": ([vp, i64, dp], c_int),
        "VecGetValuesHost": ([vp, i64, dp], c_int),
        "PCCreate": ([vp, P(vp)], c_int),
        "PCSetType": ([vp, ctypes.c_char_p], c_int),
        "PCShellSetContext": ([vp, vp], c_int),
        "PCShellGetContext": ([vp, P(vp)], c_int),
        "PCShellSetApply": ([vp, vp], c_int),
        "PCShellSetSetUp": ([vp, vp], c_int),
        "PCShellSetDestroy": ([vp, vp], c_int),
        "PCSetUp": ([vp], c_int),
        "PCApply": ([vp, vp, vp], c_int),
        "PCDestroy": ([P(vp)], c_int),
        "MatCreateFFT": ([vp, i64, P(i64), c_int, P(vp)], c_int),
        "MatMult": ([vp, vp, vp], c_int),
        "MatMultTranspose": ([vp, vp, vp], c_int),
        "MatDestroy": ([P(vp)], c_int),
        "VecPointwiseDivide": ([vp, vp, vp], c_int),
        "VecScale": ([vp, dbl, dbl], c_int),
        "applyFFT3DPrecTransport": ([vp, vp, vp], c_int),
        "setupFFTPrec3D": ([vp], c_int),
        "destroyFFTPrec3D": ([vp], c_int),
        "getFFTPrec3DContext": ([i64, dbl, i64, dbl, dbl, dbl, dbl, dbl, dbl, dbl, dbl, dbl, vp], c_int),
        "FFTPrecTransportContextCreate": ([P(vp)], c_int),
        "FFTPrecTransportContextDestroy": ([P(vp)], c_int),
        "FFTPrecTransportContextGetDims": ([vp, P(i64), dp], c_int),
        "solve_3D": ([vp, vp, vp, vp, vp, i64], c_int),
        "build_transport_col": ([vp, i64], c_int),
        "build_diag_mat_vec_3D": ([vp, vp, vp, vp, i64, i64, i64, dbl, dbl, dbl], c_int),
        "FftTransportSolver": ([i64, i64, i64, dbl, dbl, dbl, vp, vp, vp], c_int),
        "Fft3DTransportSolver": ([i64, i64, i64, dbl, dbl, dbl, dbl, dbl, dbl, dbl, vp, vp, vp], c_int),
        "Fft2DTransportSolver": ([i64, i64, dbl, dbl, dbl, dbl, dbl, vp, vp, vp], c_int),
        "Fft1DTransportSolver": ([i64, dbl, dbl, dbl, vp, vp, vp], c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
