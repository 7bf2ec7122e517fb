"""Python mirror of the reference's PETSc-facing interface, over the C ABI.

The objects are the library's PETSc stand-in (include/petsc_mini.h): ``Vec``
(device VECSEQHIP wrapping a torch tensor's memory, or host VECSEQ), ``Mat``
(FFT matrix, AIJ), ``PC`` (PCSHELL).  The functions carry the reference's names
and argument order (src/PCSHELLFft_3D.hxx, src/FftLinearSolver_3D.h), so the
parity tests read like the reference's own drivers:

    ctx = getFFTPrec3DContext(3, dt, N, ax, ay, az, xmin, ymin, zmin, xmax, ymax, zmax)
    pc = PC.shell(ctx)                        # PCSetType(PCSHELL) + PCShellSet*
    pc.setup()                                # setupFFTPrec3D
    pc.apply(b, x)                            # PCApply -> applyFFT3DPrecTransport
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np
import torch

from ._lib import CirculantError, lib
from ._lib_ext import FFTPrecTransportContext, PetscScalar, StructuredTransportContext

PETSC_COMM_WORLD = 0
PETSC_COMM_SELF = 1
PETSC_DEFAULT = -2
INSERT_VALUES, ADD_VALUES = 1, 2
NORM_1, NORM_2, NORM_INFINITY = 0, 1, 3


class PetscError(CirculantError):
    pass


def PetscCall(rc: int) -> None:
    if rc != 0:
        msg = lib().PetscErrorLastMessage().decode(errors="replace")
        cfp = lib().cfp_last_error().decode(errors="replace")
        raise PetscError(rc, f"{msg} {('| ' + cfp) if cfp else ''}".strip())


def _S(v) -> PetscScalar:
    return PetscScalar.of(v)


class Vec:
    """A PETSc Vec of the stand-in.  ``Vec.from_tensor`` wraps device memory without a copy."""

    def __init__(self, handle, keep=None, owned: bool = True):
        self.h = handle if isinstance(handle, ctypes.c_void_p) else ctypes.c_void_p(handle)
        self._keep = keep  # keeps a wrapped tensor alive
        self.owned = owned

    @classmethod
    def borrow(cls, handle) -> "Vec":
        """Non-owning view of a Vec created elsewhere (e.g. ctx.Diag made by setupFFTPrec3D)."""
        return cls(handle, owned=False)

    @classmethod
    def from_tensor(cls, t: torch.Tensor) -> "Vec":
        if t.dtype != torch.complex128 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("need a contiguous complex128 device tensor")
        h = ctypes.c_void_p()
        PetscCall(lib().VecCreateSeqHIPWithArray(PETSC_COMM_SELF, 1, t.numel(), t.data_ptr(), ctypes.byref(h)))
        return cls(h, keep=t)

    @classmethod
    def from_tensor_mpi(cls, t: torch.Tensor, N: int, comm: int = PETSC_COMM_WORLD) -> "Vec":
        """VecCreateMPIHIPWithArray: this rank's rows of a distributed Vec, in t's memory."""
        if t.dtype != torch.complex128 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("need a contiguous complex128 device tensor")
        h = ctypes.c_void_p()
        PetscCall(lib().VecCreateMPIHIPWithArray(int(comm), 1, t.numel(), int(N), t.data_ptr(), ctypes.byref(h)))
        return cls(h, keep=t)

    @classmethod
    def seq_hip(cls, n: int) -> "Vec":
        h = ctypes.c_void_p()
        PetscCall(lib().VecCreateSeqHIP(PETSC_COMM_SELF, int(n), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def seq(cls, n: int) -> "Vec":
        """Host-only VECSEQ (exercises the PCIe staging path)."""
        h = ctypes.c_void_p()
        PetscCall(lib().VecCreateSeq(PETSC_COMM_SELF, int(n), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def mpi(cls, N: int, comm: int = PETSC_COMM_WORLD, nlocal: int = -1) -> "Vec":
        """VecCreateMPI(comm, PETSC_DECIDE, N): this rank's block of rows, host memory."""
        h = ctypes.c_void_p()
        PetscCall(lib().VecCreateMPI(int(comm), int(nlocal), int(N), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def mpi_hip(cls, N: int, comm: int = PETSC_COMM_WORLD, nlocal: int = -1) -> "Vec":
        """VecCreateMPIHIP(comm, PETSC_DECIDE, N): this rank's block of rows on the device."""
        h = ctypes.c_void_p()
        PetscCall(lib().VecCreateMPIHIP(int(comm), int(nlocal), int(N), ctypes.byref(h)))
        return cls(h)

    @property
    def size(self) -> int:
        """Global size (VecGetSize)."""
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
        a = np.ascontiguousarray(np.asarray(a, dtype=np.complex128).reshape(-1))
        if a.size != self.local_size:
            raise ValueError("size mismatch")
        p = ctypes.c_void_p()
        PetscCall(lib().VecGetArray(self.h, ctypes.byref(p)))
        ctypes.memmove(p, a.ctypes.data, a.nbytes)
        PetscCall(lib().VecRestoreArray(self.h, ctypes.byref(p)))
        return self

    def array(self) -> np.ndarray:
        """This rank's rows (local size)."""
        n = self.local_size
        p = ctypes.c_void_p()
        PetscCall(lib().VecGetArrayRead(self.h, ctypes.byref(p)))
        out = np.empty(n, dtype=np.complex128)
        ctypes.memmove(out.ctypes.data, p, out.nbytes)
        PetscCall(lib().VecRestoreArrayRead(self.h, ctypes.byref(p)))
        return out

    def set(self, alpha) -> "Vec":
        PetscCall(lib().VecSet(self.h, _S(alpha)))
        return self

    def norm(self, kind: int = NORM_2) -> float:
        v = ctypes.c_double()
        PetscCall(lib().VecNorm(self.h, kind, ctypes.byref(v)))
        return v.value

    def dot(self, other: "Vec") -> complex:
        s = PetscScalar()
        PetscCall(lib().VecDot(self.h, other.h, ctypes.byref(s)))
        return complex(s)

    def axpy(self, alpha, x: "Vec") -> "Vec":
        PetscCall(lib().VecAXPY(self.h, _S(alpha), x.h))
        return self

    def scale(self, alpha) -> "Vec":
        PetscCall(lib().VecScale(self.h, _S(alpha)))
        return self

    def state(self) -> int:
        """PetscObjectStateGet: increases on every write access."""
        v = ctypes.c_int64()
        PetscCall(lib().PetscObjectStateGet(self.h, ctypes.byref(v)))
        return v.value

    def hip_array(self):
        """Context manager: VecHIPGetArray / VecHIPRestoreArray (read-write device pointer)."""
        vec = self

        class _Arr:
            def __enter__(self_):
                self_.p = ctypes.c_void_p()
                PetscCall(lib().VecHIPGetArray(vec.h, ctypes.byref(self_.p)))
                return self_.p.value

            def __exit__(self_, *exc):
                PetscCall(lib().VecHIPRestoreArray(vec.h, ctypes.byref(self_.p)))
        return _Arr()

    def destroy(self) -> None:
        if self.owned and self.h is not None and self.h.value:
            PetscCall(lib().VecDestroy(ctypes.byref(self.h)))
        self.h = None
        self._keep = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class Comm:
    """A communicator of several ranks for the stand-in PETSc (an int handle, as MPI_Comm).

    ``Comm.torch(group)``: the collectives are torch.distributed's on `group` (under gloo the
    library stages the exchange pieces through pinned host memory) -- several processes may
    then share one GPU.  ``Comm.rccl(group)``: an RCCL communicator inside the library (one
    process per GPU), its unique id broadcast over `group`.  ``set_world()`` makes it
    PETSC_COMM_WORLD, the communicator setupFFTPrec3D builds its FFT matrix on
    (src/PCSHELLFft_3D.cxx:34-35)."""

    _A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
    _RED = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int64, ctypes.c_int)

    class _Ops(ctypes.Structure):
        pass

    _Ops._fields_ = [("alltoall", _A2A), ("allreduce", _RED), ("user", ctypes.c_void_p)]

    # the ctypes callbacks of live communicators, by handle: the library calls them for as long
    # as the communicator exists, whether or not this Python object is still referenced
    _REGISTRY: dict = {}

    def __init__(self, handle: int, keep=()):
        self.handle = int(handle)
        if keep:
            Comm._REGISTRY[self.handle] = keep

    @classmethod
    def torch(cls, group=None) -> "Comm":
        import torch.distributed as dist
        size, rank = dist.get_world_size(group), dist.get_rank(group)

        def alltoall(_user, send, recv, nbytes):
            try:
                n = size * nbytes // 8
                s = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_double * n).from_address(send)))
                r = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_double * n).from_address(recv)))
                dist.all_to_all_single(r, s.clone(), group=group)
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

        a2a, red = cls._A2A(alltoall), cls._RED(allreduce)
        ops = cls._Ops(a2a, red, None)
        h = ctypes.c_int()
        PetscCall(lib().PetscMiniCommCreate(size, rank, ctypes.byref(ops), ctypes.byref(h)))
        return cls(h.value, keep=(a2a, red, ops))

    @classmethod
    def rccl(cls, group=None, device: int | None = None) -> "Comm":
        import torch.distributed as dist
        size, rank = dist.get_world_size(group), dist.get_rank(group)
        nbytes = lib().cfp_dist_unique_id_bytes()
        uid = ctypes.create_string_buffer(nbytes)
        if rank == 0:
            from ._lib import check
            check(lib().cfp_dist_get_unique_id(uid))
        t = torch.frombuffer(bytearray(uid.raw), dtype=torch.uint8).clone()
        if dist.get_backend(group) == "nccl":
            t = t.to(f"cuda:{torch.cuda.current_device() if device is None else device}")
        dist.broadcast(t, src=0, group=group)
        uid = ctypes.create_string_buffer(bytes(t.cpu().numpy().tobytes()), nbytes)
        h = ctypes.c_int()
        PetscCall(lib().PetscMiniCommCreateRCCL(size, rank, uid, ctypes.byref(h)))
        return cls(h.value)

    @property
    def size(self) -> int:
        v = ctypes.c_int()
        lib().MPI_Comm_size(self.handle, ctypes.byref(v))
        return v.value

    @property
    def rank(self) -> int:
        v = ctypes.c_int()
        lib().MPI_Comm_rank(self.handle, ctypes.byref(v))
        return v.value

    def set_world(self) -> "Comm":
        PetscCall(lib().PetscMiniSetCommWorld(self.handle))
        return self

    def allreduce(self, values, op: int = 0) -> np.ndarray:
        a = np.ascontiguousarray(np.asarray(values, dtype=np.float64).reshape(-1))
        PetscCall(lib().PetscMiniAllreduce(self.handle, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.size,
                                           int(op)))
        return a

    def destroy(self) -> None:
        """PetscMiniCommDestroy; refused (PetscError) while FFT matrices built on it exist."""
        if self.handle >= 2:
            h = ctypes.c_int(self.handle)
            PetscCall(lib().PetscMiniCommDestroy(ctypes.byref(h)))
            Comm._REGISTRY.pop(self.handle, None)
        self.handle = PETSC_COMM_SELF


def set_comm_world(comm: "Comm | int") -> None:
    """PETSC_COMM_WORLD := comm (PETSC_COMM_SELF: back to one rank)."""
    PetscCall(lib().PetscMiniSetCommWorld(comm.handle if isinstance(comm, Comm) else int(comm)))


class Mat:
    def __init__(self, handle: ctypes.c_void_p, owned: bool = True):
        self.h = handle
        self.owned = owned

    @classmethod
    def create_fft(cls, dims: Sequence[int]) -> "Mat":
        """MatCreateFFT(comm, ndim, dims = {n_z, n_y, n_x}, MATFFTW, &A)."""
        d = (ctypes.c_int64 * len(dims))(*[int(v) for v in dims])
        h = ctypes.c_void_p()
        PetscCall(lib().MatCreateFFT(PETSC_COMM_WORLD, len(dims), d, b"fftw", ctypes.byref(h)))
        return cls(h)

    @classmethod
    def aij(cls, rowptr, col, val, shape) -> "Mat":
        m, n = shape
        rp = np.ascontiguousarray(rowptr, dtype=np.int64)
        cj = np.ascontiguousarray(col, dtype=np.int64)
        va = np.ascontiguousarray(val, dtype=np.complex128)
        h = ctypes.c_void_p()
        PetscCall(lib().MatCreateSeqAIJWithArrays(PETSC_COMM_SELF, m, n,
                                                  rp.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                  cj.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                  va.ctypes.data, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def create_aij(cls, N: int, comm: int = PETSC_COMM_WORLD, nlocal: int = -1) -> "Mat":
        """MatCreateAIJ(comm, nlocal | PETSC_DECIDE, same, N, N, ...): an N x N matrix to fill with
        set_values and assemble (the reference's MatCreateAIJ on PETSC_COMM_WORLD)."""
        h = ctypes.c_void_p()
        PetscCall(lib().MatCreateAIJ(comm, nlocal, nlocal, N, N, 7, None, 6, None, ctypes.byref(h)))
        return cls(h)

    def set_values(self, rows, cols, vals, add: bool = False) -> "Mat":
        """MatSetValues(A, len(rows), rows, len(cols), cols, vals (row-major), mode)."""
        r = np.ascontiguousarray(rows, dtype=np.int64)
        c = np.ascontiguousarray(cols, dtype=np.int64)
        v = np.ascontiguousarray(vals, dtype=np.complex128).reshape(-1)
        if v.size != r.size * c.size:
            raise ValueError("vals must hold len(rows) * len(cols) values")
        PetscCall(lib().MatSetValues(self.h, r.size, r.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), c.size,
                                     c.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), v.ctypes.data,
                                     ADD_VALUES if add else INSERT_VALUES))
        return self

    def assemble(self) -> "Mat":
        PetscCall(lib().MatAssemblyBegin(self.h, 0))
        PetscCall(lib().MatAssemblyEnd(self.h, 0))
        return self

    def ownership_range(self) -> tuple:
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        PetscCall(lib().MatGetOwnershipRange(self.h, ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    def halo(self) -> tuple:
        """(ghost columns of this rank, the largest per-peer halo over the ranks): MATMPIAIJ."""
        g, m = ctypes.c_int64(), ctypes.c_int64()
        PetscCall(lib().PetscMiniMatMPIAIJGetHalo(self.h, ctypes.byref(g), ctypes.byref(m)))
        return g.value, m.value

    def create_vecs(self, nvec: int = 1) -> list:
        hs = [ctypes.c_void_p() for _ in range(3)]
        refs = [ctypes.byref(hs[i]) if i < nvec else None for i in range(3)]
        PetscCall(lib().MatCreateVecsFFTW(self.h, *refs))
        return [Vec(hs[i]) for i in range(nvec)]

    def solve_counts(self) -> tuple:
        """(solve_3D calls that used the plan's own symbol, calls that streamed the given Diag)."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        PetscCall(lib().MatFFTHIPGetSolveCounts(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def mult(self, x: Vec, y: Vec) -> Vec:
        PetscCall(lib().MatMult(self.h, x.h, y.h))
        return y

    def mult_transpose(self, x: Vec, y: Vec) -> Vec:
        PetscCall(lib().MatMultTranspose(self.h, x.h, y.h))
        return y

    def aij_format(self) -> str:
        """The stand-in AIJ's device storage: 'dia' (row-class diagonal form), 'bdia' (block
        row-class form, e.g. the interleaved wave operator), 'csr', or 'none' before the first
        device MatMult."""
        f = ctypes.c_int()
        PetscCall(lib().PetscMiniMatAIJGetFormat(self.h, ctypes.byref(f)))
        return {1: "dia", 2: "bdia", 0: "csr"}.get(f.value, "none")

    def shift(self, a) -> "Mat":
        PetscCall(lib().MatShift(self.h, _S(a)))
        return self

    def destroy(self) -> None:
        if self.owned and self.h is not None and self.h.value:
            PetscCall(lib().MatDestroy(ctypes.byref(self.h)))
        self.h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class FFTPrecWaveContext(ctypes.Structure):
    """struct FFTPrecWaveContext (include/wave_system.h)."""
    _fields_ = [("n_x", ctypes.c_int64), ("n_y", ctypes.c_int64), ("n_z", ctypes.c_int64),
                ("kappa_x", ctypes.c_double), ("kappa_y", ctypes.c_double), ("kappa_z", ctypes.c_double),
                ("c0", ctypes.c_double), ("plan", ctypes.c_void_p), ("dim", ctypes.c_int64)]


def _fn(name: str) -> int:
    return ctypes.cast(getattr(lib(), name), ctypes.c_void_p).value


class PC:
    def __init__(self, handle: ctypes.c_void_p | None = None, owned: bool = True):
        if handle is None:
            handle = ctypes.c_void_p()
            PetscCall(lib().PCCreate(PETSC_COMM_WORLD, ctypes.byref(handle)))
        self.h = handle
        self.owned = owned
        self.ctx = None

    @classmethod
    def shell(cls, ctx: FFTPrecTransportContext) -> "PC":
        """PCSetType(pc, PCSHELL); PCShellSetContext; PCShellSetSetUp/Apply/Destroy with the
        reference's callbacks (the registration the reference never does, ToDo.md:1)."""
        return cls().set_shell(ctx)

    def set_shell(self, ctx: FFTPrecTransportContext) -> "PC":
        PetscCall(lib().PCSetType(self.h, b"shell"))
        self.ctx = ctx
        PetscCall(lib().PCShellSetContext(self.h, ctypes.addressof(ctx)))
        PetscCall(lib().PCShellSetSetUp(self.h, _fn("setupFFTPrec3D")))
        PetscCall(lib().PCShellSetApply(self.h, _fn("applyFFT3DPrecTransport")))
        PetscCall(lib().PCShellSetDestroy(self.h, _fn("destroyFFTPrec3D")))
        return self

    @classmethod
    def wave_shell(cls, ctx: "FFTPrecWaveContext") -> "PC":
        """PCSHELL with the block-circulant wave callbacks (include/wave_system.h):
        setupFFTPrec3DWave / applyFFT3DPrecWave / destroyFFTPrec3DWave."""
        pc = cls()
        PetscCall(lib().PCSetType(pc.h, b"shell"))
        pc.ctx = ctx
        PetscCall(lib().PCShellSetContext(pc.h, ctypes.addressof(ctx)))
        PetscCall(lib().PCShellSetSetUp(pc.h, _fn("setupFFTPrec3DWave")))
        PetscCall(lib().PCShellSetApply(pc.h, _fn("applyFFT3DPrecWave")))
        PetscCall(lib().PCShellSetDestroy(pc.h, _fn("destroyFFTPrec3DWave")))
        return pc

    @classmethod
    def none(cls) -> "PC":
        return cls().set_none()

    def set_none(self) -> "PC":
        PetscCall(lib().PCSetType(self.h, b"none"))
        return self

    def setup(self) -> "PC":
        PetscCall(lib().PCSetUp(self.h))
        return self

    def apply(self, b: Vec, x: Vec) -> Vec:
        PetscCall(lib().PCApply(self.h, b.h, x.h))
        return x

    def destroy(self) -> None:
        if self.owned and self.h is not None and self.h.value:
            PetscCall(lib().PCDestroy(ctypes.byref(self.h)))
        self.h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


KSP_REASONS = {0: "ITERATING", 2: "CONVERGED_RTOL", 3: "CONVERGED_ATOL", 4: "CONVERGED_ITS",
               7: "CONVERGED_HAPPY_BREAKDOWN", -3: "DIVERGED_ITS", -4: "DIVERGED_DTOL", -5: "DIVERGED_BREAKDOWN"}
PC_LEFT, PC_RIGHT = 0, 1


class KSP:
    """KSPGMRES of the stand-in (csrc/ksp_gmres.cpp): restart 30, left preconditioning, CGS,
    rtol 1e-5 / abstol 1e-50 / dtol 1e5 / maxits 10000 unless set, as PETSc's defaults."""

    def __init__(self):
        self.h = ctypes.c_void_p()
        PetscCall(lib().KSPCreate(PETSC_COMM_WORLD, ctypes.byref(self.h)))
        PetscCall(lib().KSPSetType(self.h, b"gmres"))
        self._ops = None
        self._pc = None

    def set_type(self, t: str) -> "KSP":
        PetscCall(lib().KSPSetType(self.h, t.encode()))
        return self

    def set_tolerances(self, rtol=PETSC_DEFAULT, abstol=PETSC_DEFAULT, dtol=PETSC_DEFAULT,
                       maxits=PETSC_DEFAULT) -> "KSP":
        PetscCall(lib().KSPSetTolerances(self.h, float(rtol), float(abstol), float(dtol), int(maxits)))
        return self

    def set_restart(self, m: int) -> "KSP":
        PetscCall(lib().KSPGMRESSetRestart(self.h, int(m)))
        return self

    def set_pc_side(self, side: int) -> "KSP":
        PetscCall(lib().KSPSetPCSide(self.h, int(side)))
        return self

    def set_initial_guess_nonzero(self, flag: bool = True) -> "KSP":
        PetscCall(lib().KSPSetInitialGuessNonzero(self.h, 1 if flag else 0))
        return self

    def get_pc(self) -> PC:
        if self._pc is None:
            h = ctypes.c_void_p()
            PetscCall(lib().KSPGetPC(self.h, ctypes.byref(h)))
            self._pc = PC(h, owned=False)
        return self._pc

    def set_operators(self, A: Mat, P: Mat | None = None) -> "KSP":
        self._ops = (A, P or A)
        PetscCall(lib().KSPSetOperators(self.h, A.h, (P or A).h))
        return self

    def setup(self) -> "KSP":
        PetscCall(lib().KSPSetUp(self.h))
        return self

    def solve(self, b: Vec, x: Vec) -> int:
        PetscCall(lib().KSPSolve(self.h, b.h, x.h))
        return self.reason

    @property
    def reason(self) -> int:
        r = ctypes.c_int()
        PetscCall(lib().KSPGetConvergedReason(self.h, ctypes.byref(r)))
        return r.value

    @property
    def its(self) -> int:
        n = ctypes.c_int64()
        PetscCall(lib().KSPGetIterationNumber(self.h, ctypes.byref(n)))
        return n.value

    @property
    def rnorm(self) -> float:
        r = ctypes.c_double()
        PetscCall(lib().KSPGetResidualNorm(self.h, ctypes.byref(r)))
        return r.value

    def pc_stats(self) -> tuple:
        n, s = ctypes.c_int64(), ctypes.c_double()
        PetscCall(lib().KSPMiniGetPCApplyStats(self.h, ctypes.byref(n), ctypes.byref(s)))
        return n.value, s.value

    def destroy(self) -> None:
        if self.h is not None and self.h.value:
            if self._pc is not None:
                self._pc.h = None
            PetscCall(lib().KSPDestroy(ctypes.byref(self.h)))
        self.h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ------------------------------------------------------------- reference-named functions
def getFFTPrec3DContext(ndim, dt, nbCells, a_x, a_y, a_z, Xmin, Ymin, Zmin, Xmax, Ymax, Zmax
                        ) -> FFTPrecTransportContext:
    """src/PCSHELLFft_3D.cxx:101-151 (returns the filled context)."""
    ctx = FFTPrecTransportContext()
    PetscCall(lib().getFFTPrec3DContext(int(ndim), _S(dt), int(nbCells), _S(a_x), _S(a_y), _S(a_z), _S(Xmin),
                                        _S(Ymin), _S(Zmin), _S(Xmax), _S(Ymax), _S(Zmax), ctypes.byref(ctx)))
    return ctx


def make_context(dims: Sequence[int], lam: Sequence, space_dim: int = 3) -> FFTPrecTransportContext:
    """Context with explicit n and lambda (the reference struct filled by hand)."""
    ctx = FFTPrecTransportContext()
    ctx.spaceDim = space_dim
    ctx.n_x, ctx.n_y, ctx.n_z = (int(d) for d in dims)
    ctx.lambda_x, ctx.lambda_y, ctx.lambda_z = (PetscScalar.of(v) for v in lam)
    PetscCall(lib().FFTPrecTransportContextSetRemapBack(ctypes.byref(ctx), None))  # fresh side-table entry
    return ctx


def context_plan(ctx: FFTPrecTransportContext) -> int:
    """The HIP plan behind ctx.FFT_MAT after setupFFTPrec3D (MatFFTHIPGetPlan), as an int handle."""
    if not ctx.FFT_MAT:
        return 0
    h = ctypes.c_void_p()
    PetscCall(lib().MatFFTHIPGetPlan(ctypes.c_void_p(ctx.FFT_MAT), ctypes.byref(h)))
    return h.value or 0


def context_remap_back(ctx: FFTPrecTransportContext) -> int:
    """This build's Cartesian -> mesh remap of ctx (side table; 0 = none)."""
    h = ctypes.c_void_p()
    PetscCall(lib().FFTPrecTransportContextGetRemapBack(ctypes.byref(ctx), ctypes.byref(h)))
    return h.value or 0


def applyFFT3DPrecTransport(pc: PC, b: Vec, x: Vec) -> None:
    PetscCall(lib().applyFFT3DPrecTransport(pc.h, b.h, x.h))


def setupFFTPrec3D(pc: PC) -> None:
    PetscCall(lib().setupFFTPrec3D(pc.h))


def destroyFFTPrec3D(pc: PC) -> None:
    PetscCall(lib().destroyFFTPrec3D(pc.h))


def solve_3D(FFT_MAT: Mat, X: Vec, Diag: Vec, b: Vec, b_hat: Vec | None, size: int) -> None:
    PetscCall(lib().solve_3D(FFT_MAT.h, X.h, Diag.h, b.h, b_hat.h if b_hat is not None else None, int(size)))


def build_transport_col(c: Vec, size: int) -> None:
    PetscCall(lib().build_transport_col(c.h, int(size)))


def build_diag_mat_vec_3D(Diag: Vec, c_x_hat: Vec, c_y_hat: Vec, c_z_hat: Vec, n_x, n_y, n_z, lambda_x, lambda_y,
                          lambda_z) -> None:
    PetscCall(lib().build_diag_mat_vec_3D(Diag.h, c_x_hat.h, c_y_hat.h, c_z_hat.h, int(n_x), int(n_y), int(n_z),
                                          _S(lambda_x), _S(lambda_y), _S(lambda_z)))


def FftTransportSolver(n_x, n_y, n_z, lambda_x, lambda_y, lambda_z, X: Vec, b: Vec, FFT_MAT: Mat) -> None:
    PetscCall(lib().FftTransportSolver(int(n_x), int(n_y), int(n_z), _S(lambda_x), _S(lambda_y), _S(lambda_z),
                                       X.h, b.h, FFT_MAT.h))


def Fft3DTransportSolver(n_x, n_y, n_z, a_x, a_y, a_z, dt, delta_x, delta_y, delta_z, X: Vec, b: Vec,
                         FFT_MAT: Mat) -> None:
    PetscCall(lib().Fft3DTransportSolver(int(n_x), int(n_y), int(n_z), _S(a_x), _S(a_y), _S(a_z), _S(dt),
                                         _S(delta_x), _S(delta_y), _S(delta_z), X.h, b.h, FFT_MAT.h))


def Fft2DTransportSolver(n_x, n_y, a_x, a_y, dt, delta_x, delta_y, X: Vec, b: Vec, FFT_MAT: Mat) -> None:
    PetscCall(lib().Fft2DTransportSolver(int(n_x), int(n_y), _S(a_x), _S(a_y), _S(dt), _S(delta_x), _S(delta_y),
                                         X.h, b.h, FFT_MAT.h))


def Fft1DTransportSolver(n_x, a_x, dt, delta_x, X: Vec, b: Vec, FFT_MAT: Mat) -> None:
    PetscCall(lib().Fft1DTransportSolver(int(n_x), _S(a_x), _S(dt), _S(delta_x), X.h, b.h, FFT_MAT.h))


def StructuredContext(n_x, n_y, n_z, a_x, a_y, a_z, dt, delta_x, delta_y, delta_z, FFT_MAT: Mat
                      ) -> StructuredTransportContext:
    c = StructuredTransportContext()
    c.n_x, c.n_y, c.n_z = int(n_x), int(n_y), int(n_z)
    for name, v in (("a_x", a_x), ("a_y", a_y), ("a_z", a_z), ("dt", dt), ("delta_x", delta_x),
                    ("delta_y", delta_y), ("delta_z", delta_z)):
        setattr(c, name, PetscScalar.of(v))
    c.FFT_MAT = FFT_MAT.h
    return c


def PetscFft3DTransportSolver(customCtx: StructuredTransportContext, b: Vec, x: Vec) -> None:
    PetscCall(lib().PetscFft3DTransportSolver(customCtx, b.h, x.h))
