"""The real-scalar PETSc boundary (PetscScalar = double): ``libcirculant_fft_real.so``.

The same PETSc-named entry points as ``petsc.py`` (include/pcshell_fft3d.h, include/petsc_mini.h)
built with -DCFP_REAL_SCALAR: a PETSc configured with real scalars, which is what the
reference's ``#if !defined(PETSC_USE_COMPLEX)`` branches compile against
(src/FftLinearSolver_3D.c:6-78, 166-190).  Vecs hold doubles; FFT_MAT maps the N reals of the
grid to FFTW's r2c half spectrum ([nz][ny][nx/2 + 1] complex as interleaved reals), which is
also the layout of Diag and b_hat (pcshell_fft3d_real.cpp).

The library is loaded with RTLD_LOCAL and linked -Bsymbolic, so it coexists with the complex
``libcirculant_fft.so`` in one process (the tests load both).  No CPU fallback: a missing
library raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from ._lib import CirculantError

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libcirculant_fft_real.so")
_lock = threading.Lock()
_lib = None

PETSC_COMM_WORLD, PETSC_COMM_SELF = 0, 1
INSERT_VALUES, ADD_VALUES = 1, 2
NORM_2 = 1
MATOP_MULT = 0


class FFTPrecTransportContext(ctypes.Structure):
    """src/PCSHELLFft_3D.hxx:8-21 with PetscScalar = double."""
    _fields_ = [("spaceDim", ctypes.c_int64), ("n_x", ctypes.c_int64), ("n_y", ctypes.c_int64),
                ("n_z", ctypes.c_int64), ("lambda_x", ctypes.c_double), ("lambda_y", ctypes.c_double),
                ("lambda_z", ctypes.c_double), ("FFT_MAT", ctypes.c_void_p), ("intersectionMatrix", ctypes.c_void_p),
                ("Diag", ctypes.c_void_p), ("b_hat", ctypes.c_void_p), ("b_cartesien", ctypes.c_void_p)]


class StructuredTransportContext(ctypes.Structure):
    """src/FftLinearSolver_3D.h:7-19 with PetscScalar = double (passed by value)."""
    _fields_ = [("n_x", ctypes.c_int64), ("n_y", ctypes.c_int64), ("n_z", ctypes.c_int64),
                ("a_x", ctypes.c_double), ("a_y", ctypes.c_double), ("a_z", ctypes.c_double), ("dt", ctypes.c_double),
                ("delta_x", ctypes.c_double), ("delta_y", ctypes.c_double), ("delta_z", ctypes.c_double),
                ("FFT_MAT", ctypes.c_void_p)]


def _declare(L) -> None:
    vp, i64, c_int, d = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
    P = ctypes.POINTER
    sig = {
        "PetscErrorLastMessage": ([], ctypes.c_char_p),
        "VecCreateSeq": ([c_int, i64, P(vp)], c_int),
        "VecCreateSeqHIP": ([c_int, i64, P(vp)], c_int),
        "VecCreateMPI": ([c_int, i64, i64, P(vp)], c_int),
        "VecCreateMPIHIP": ([c_int, i64, i64, P(vp)], c_int),
        "VecGetLocalSize": ([vp, P(i64)], c_int),
        "VecGetOwnershipRange": ([vp, P(i64), P(i64)], c_int),
        "PetscMiniCommCreate": ([c_int, c_int, vp, P(c_int)], c_int),
        "PetscMiniCommDestroy": ([P(c_int)], c_int),
        "PetscMiniSetCommWorld": ([c_int], c_int),
        "MatFFTHIPGetDistPlan": ([vp, P(vp)], c_int),
        "VecDestroy": ([P(vp)], c_int),
        "VecGetSize": ([vp, P(i64)], c_int),
        "VecGetArray": ([vp, P(vp)], c_int),
        "VecRestoreArray": ([vp, P(vp)], c_int),
        "VecGetArrayRead": ([vp, P(vp)], c_int),
        "VecRestoreArrayRead": ([vp, P(vp)], c_int),
        "VecSet": ([vp, d], c_int),
        "VecScale": ([vp, d], c_int),
        "VecCopy": ([vp, vp], c_int),
        "VecNorm": ([vp, c_int, P(d)], c_int),
        "VecDot": ([vp, vp, P(d)], c_int),
        "VecAXPY": ([vp, d, vp], c_int),
        "MatCreateFFT": ([c_int, i64, P(i64), ctypes.c_char_p, P(vp)], c_int),
        "MatCreateVecsFFTW": ([vp, P(vp), P(vp), P(vp)], c_int),
        "MatCreateSeqAIJWithArrays": ([c_int, i64, i64, P(i64), P(i64), P(d), P(vp)], c_int),
        "MatShift": ([vp, d], c_int),
        "MatMult": ([vp, vp, vp], c_int),
        "MatMultTranspose": ([vp, vp, vp], c_int),
        "MatDestroy": ([P(vp)], c_int),
        "MatFFTHIPGetRealPlan": ([vp, P(vp)], c_int),
        "MatFFTHIPGetSolveCounts": ([vp, P(i64), P(i64)], c_int),
        "PCCreate": ([c_int, P(vp)], c_int),
        "PCSetType": ([vp, ctypes.c_char_p], c_int),
        "PCShellSetContext": ([vp, vp], c_int),
        "PCShellSetSetUp": ([vp, vp], c_int),
        "PCShellSetApply": ([vp, vp], c_int),
        "PCShellSetDestroy": ([vp, vp], c_int),
        "PCSetUp": ([vp], c_int),
        "PCApply": ([vp, vp, vp], c_int),
        "PCDestroy": ([P(vp)], c_int),
        "KSPCreate": ([c_int, P(vp)], c_int),
        "KSPSetType": ([vp, ctypes.c_char_p], c_int),
        "KSPSetOperators": ([vp, vp, vp], c_int),
        "KSPGetPC": ([vp, P(vp)], c_int),
        "KSPSetTolerances": ([vp, d, d, d, i64], c_int),
        "KSPSolve": ([vp, vp, vp], c_int),
        "KSPGetIterationNumber": ([vp, P(i64)], c_int),
        "KSPGetConvergedReason": ([vp, P(c_int)], c_int),
        "KSPDestroy": ([P(vp)], c_int),
        "solve_3D": ([vp, vp, vp, vp, vp, i64], c_int),
        "build_transport_col": ([vp, i64], c_int),
        "build_diag_mat_vec_3D": ([vp, vp, vp, vp, i64, i64, i64, d, d, d], c_int),
        "PetscFft3DTransportSolver": ([StructuredTransportContext, vp, vp], c_int),
        "setupFFTPrec3D": ([vp], c_int),
        "destroyFFTPrec3D": ([vp], c_int),
        "applyFFT3DPrecTransport": ([vp, vp, vp], c_int),
        "getFFTPrec3DContext": ([i64, d, i64, d, d, d, d, d, d, d, d, d, P(FFTPrecTransportContext)], c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res


def lib():
    """Load libcirculant_fft_real.so (raises if missing: no CPU fallback)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(f"libcirculant_fft_real.so not found at {LIB_PATH}; build it with "
                                      "`make -C circulantpreconditioner_amd/csrc`")
                L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
                _declare(L)
                _lib = L
    return _lib


class PetscError(CirculantError):
    pass


def PetscCall(rc: int) -> None:
    if rc != 0:
        msg = lib().PetscErrorLastMessage()
        raise PetscError(rc, msg.decode(errors="replace") if msg else "")


def fn(name: str) -> int:
    """Address of a library function (for PCShellSetApply & co.)."""
    return ctypes.cast(getattr(lib(), name), ctypes.c_void_p).value


class Vec:
    """A real Vec (host VECSEQ or device VECSEQHIP) of the real-scalar stand-in."""

    def __init__(self, h: ctypes.c_void_p):
        self.h = h

    @classmethod
    def seq(cls, n: int, hip: bool = False) -> "Vec":
        h = ctypes.c_void_p()
        PetscCall((lib().VecCreateSeqHIP if hip else lib().VecCreateSeq)(PETSC_COMM_SELF, int(n), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def mpi(cls, N: int, hip: bool = False, nlocal: int = -1, comm: int = PETSC_COMM_WORLD) -> "Vec":
        """VecCreateMPI(HIP)(comm, PETSC_DECIDE or nlocal, N): this rank's block of rows."""
        h = ctypes.c_void_p()
        PetscCall((lib().VecCreateMPIHIP if hip else lib().VecCreateMPI)(int(comm), int(nlocal), int(N),
                                                                          ctypes.byref(h)))
        return cls(h)

    @property
    def size(self) -> int:
        n = ctypes.c_int64()
        PetscCall(lib().VecGetSize(self.h, ctypes.byref(n)))
        return n.value

    @property
    def local_size(self) -> int:
        n = ctypes.c_int64()
        PetscCall(lib().VecGetLocalSize(self.h, ctypes.byref(n)))
        return n.value

    def ownership_range(self) -> tuple:
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        PetscCall(lib().VecGetOwnershipRange(self.h, ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    def set_array(self, a) -> "Vec":
        """Write this rank's rows (local size)."""
        a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
        assert a.size == self.local_size
        p = ctypes.c_void_p()
        PetscCall(lib().VecGetArray(self.h, ctypes.byref(p)))
        ctypes.memmove(p.value, a.ctypes.data, a.nbytes)
        PetscCall(lib().VecRestoreArray(self.h, ctypes.byref(p)))
        return self

    def array(self) -> np.ndarray:
        """This rank's rows (local size)."""
        n = self.local_size
        p = ctypes.c_void_p()
        PetscCall(lib().VecGetArrayRead(self.h, ctypes.byref(p)))
        out = np.ctypeslib.as_array((ctypes.c_double * n).from_address(p.value)).copy()
        PetscCall(lib().VecRestoreArrayRead(self.h, ctypes.byref(p)))
        return out

    def destroy(self) -> None:
        if self.h is not None and self.h.value:
            PetscCall(lib().VecDestroy(ctypes.byref(self.h)))
        self.h = None


class Comm:
    """A communicator of several ranks for the real-scalar stand-in (its own communicator table:
    the library is loaded RTLD_LOCAL), with torch.distributed's collectives on `group` -- the
    counterpart of petsc.Comm.torch.  set_world() makes it PETSC_COMM_WORLD."""

    _A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
    _RED = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int64,
                            ctypes.c_int)

    class _Ops(ctypes.Structure):
        pass

    _Ops._fields_ = [("alltoall", _A2A), ("allreduce", _RED), ("user", ctypes.c_void_p)]
    _REGISTRY: dict = {}  # callbacks of live communicators, by handle

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        size, rank = dist.get_world_size(group), dist.get_rank(group)

        def alltoall(_user, send, recv, nbytes):
            try:
                n = size * nbytes // 8
                s_ = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_double * n).from_address(send)))
                r_ = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_double * n).from_address(recv)))
                dist.all_to_all_single(r_, s_.clone(), group=group)
                return 0
            except Exception:  # reported to the library as a failed collective
                return 1

        def allreduce(_user, buf, count, op):
            try:
                a = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_double * count).from_address(
                    ctypes.addressof(buf.contents))))
                t = a.clone()
                dist.all_reduce(t, op=dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.SUM, group=group)
                a.copy_(t)
                return 0
            except Exception:
                return 1

        a2a, red = self._A2A(alltoall), self._RED(allreduce)
        ops = self._Ops(a2a, red, None)
        h = ctypes.c_int()
        PetscCall(lib().PetscMiniCommCreate(size, rank, ctypes.byref(ops), ctypes.byref(h)))
        self.handle = h.value
        Comm._REGISTRY[self.handle] = (a2a, red, ops)

    def set_world(self) -> "Comm":
        PetscCall(lib().PetscMiniSetCommWorld(self.handle))
        return self

    def destroy(self) -> None:
        h = ctypes.c_int(self.handle)
        PetscCall(lib().PetscMiniCommDestroy(ctypes.byref(h)))
        Comm._REGISTRY.pop(self.handle, None)


def set_comm_world(handle: int) -> None:
    PetscCall(lib().PetscMiniSetCommWorld(int(handle)))


def mat_create_fft(dims) -> ctypes.c_void_p:
    """MatCreateFFT(PETSC_COMM_WORLD, ndim, dims = {n_z, n_y, n_x} row-major, MATFFTW)."""
    arr = (ctypes.c_int64 * len(dims))(*[int(v) for v in dims])
    A = ctypes.c_void_p()
    PetscCall(lib().MatCreateFFT(PETSC_COMM_WORLD, len(dims), arr, b"fftw", ctypes.byref(A)))
    return A


def mat_create_vecs_fftw(A) -> tuple:
    x, y, z = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    PetscCall(lib().MatCreateVecsFFTW(A, ctypes.byref(x), ctypes.byref(y), ctypes.byref(z)))
    return Vec(x), Vec(y), Vec(z)


def mat_aij(A_csr) -> ctypes.c_void_p:
    """MatCreateSeqAIJWithArrays from a real scipy CSR matrix."""
    ip = np.ascontiguousarray(A_csr.indptr.astype(np.int64))
    jp = np.ascontiguousarray(A_csr.indices.astype(np.int64))
    v = np.ascontiguousarray(A_csr.data.astype(np.float64))
    M = ctypes.c_void_p()
    PetscCall(lib().MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, A_csr.shape[0], A_csr.shape[1],
                                              ip.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                              jp.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                              v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(M)))
    return M


def pc_shell(ctx: FFTPrecTransportContext) -> ctypes.c_void_p:
    """PCSHELL registered as ToDo.md:1 intends: context + setup / apply / destroy callbacks."""
    pc = ctypes.c_void_p()
    L = lib()
    PetscCall(L.PCCreate(PETSC_COMM_WORLD, ctypes.byref(pc)))
    PetscCall(L.PCSetType(pc, b"shell"))
    PetscCall(L.PCShellSetContext(pc, ctypes.addressof(ctx)))
    PetscCall(L.PCShellSetSetUp(pc, fn("setupFFTPrec3D")))
    PetscCall(L.PCShellSetApply(pc, fn("applyFFT3DPrecTransport")))
    PetscCall(L.PCShellSetDestroy(pc, fn("destroyFFTPrec3D")))
    PetscCall(L.PCSetUp(pc))
    return pc
