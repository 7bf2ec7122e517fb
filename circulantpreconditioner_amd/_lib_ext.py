"""ctypes signatures of the slab-distributed plan (include/circulant_fft_dist.h) and of
the PETSc PCSHELL boundary (include/pcshell_fft3d.h, include/petsc_mini.h)."""
from __future__ import annotations

import ctypes


class PetscScalar(ctypes.Structure):
    """PetscScalar of a complex PETSc build (std::complex<double> / double _Complex)."""
    _fields_ = [("re", ctypes.c_double), ("im", ctypes.c_double)]

    @classmethod
    def of(cls, v) -> "PetscScalar":
        c = complex(v)
        return cls(c.real, c.imag)

    def __complex__(self):
        return complex(self.re, self.im)


class FFTPrecTransportContext(ctypes.Structure):
    """struct FFTPrecTransportContext, the reference's exact 12 members (src/PCSHELLFft_3D.hxx:8-21);
    this build's additions live in a side table (FFTPrecTransportContextSetRemapBack) and the
    plan behind FFT_MAT (MatFFTHIPGetPlan)."""
    _fields_ = [("spaceDim", ctypes.c_int64), ("n_x", ctypes.c_int64), ("n_y", ctypes.c_int64),
                ("n_z", ctypes.c_int64), ("lambda_x", PetscScalar), ("lambda_y", PetscScalar),
                ("lambda_z", PetscScalar), ("FFT_MAT", ctypes.c_void_p), ("intersectionMatrix", ctypes.c_void_p),
                ("Diag", ctypes.c_void_p), ("b_hat", ctypes.c_void_p), ("b_cartesien", ctypes.c_void_p)]


class StructuredTransportContext(ctypes.Structure):
    """struct StructuredTransportContext (src/FftLinearSolver_3D.h:7-19), passed by value."""
    _fields_ = [("n_x", ctypes.c_int64), ("n_y", ctypes.c_int64), ("n_z", ctypes.c_int64),
                ("a_x", PetscScalar), ("a_y", PetscScalar), ("a_z", PetscScalar), ("dt", PetscScalar),
                ("delta_x", PetscScalar), ("delta_y", PetscScalar), ("delta_z", PetscScalar),
                ("FFT_MAT", ctypes.c_void_p)]


class TransportConfig(ctypes.Structure):
    """cfp_transport_config (include/transport_equation.h)."""
    _fields_ = [("nx", ctypes.c_int64), ("ny", ctypes.c_int64), ("nz", ctypes.c_int64),
                ("xmin", ctypes.c_double * 3), ("xmax", ctypes.c_double * 3), ("a", ctypes.c_double * 3),
                ("cfl", ctypes.c_double), ("tmax", ctypes.c_double), ("ntmax", ctypes.c_int64),
                ("precision", ctypes.c_double), ("max_its", ctypes.c_int64), ("restart", ctypes.c_int64),
                ("pc", ctypes.c_int), ("sign_mode", ctypes.c_int), ("lambda_mode", ctypes.c_int),
                ("pc_side", ctypes.c_int), ("on_device", ctypes.c_int), ("fuse", ctypes.c_int),
                ("profile", ctypes.c_int)]


class TransportResult(ctypes.Structure):
    """cfp_transport_result (include/transport_equation.h)."""
    _fields_ = [("steps", ctypes.c_int64), ("dt", ctypes.c_double), ("time", ctypes.c_double),
                ("total_its", ctypes.c_int64), ("max_step_its", ctypes.c_int64), ("min_step_its", ctypes.c_int64),
                ("last_reason", ctypes.c_int), ("all_converged", ctypes.c_int), ("last_residual", ctypes.c_double),
                ("last_norm_dU", ctypes.c_double), ("solve_seconds", ctypes.c_double),
                ("pc_seconds", ctypes.c_double), ("pc_calls", ctypes.c_int64), ("setup_seconds", ctypes.c_double),
                ("lambda_", ctypes.c_double * 3), ("loop_seconds", ctypes.c_double), ("dev_ms_", ctypes.c_double * 4),
                ("dev_launches_", ctypes.c_int64 * 4), ("fused_dots", ctypes.c_int64), ("fused_norms", ctypes.c_int64),
                ("rstart", ctypes.c_int64), ("nlocal", ctypes.c_int64)]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if not k.endswith("_")}
        d["lambda"] = list(self.lambda_)
        d["dev_ms"] = dict(zip(("pcapply", "matmult", "vector", "copy"), self.dev_ms_))
        d["dev_launches"] = dict(zip(("pcapply", "matmult", "vector", "copy"), self.dev_launches_))
        return d


class WaveConfig(ctypes.Structure):
    """cfp_wave_config (include/wave_system.h)."""
    _fields_ = [("nx", ctypes.c_int64), ("ny", ctypes.c_int64), ("nz", ctypes.c_int64),
                ("xmin", ctypes.c_double * 3), ("xmax", ctypes.c_double * 3), ("c0", ctypes.c_double),
                ("cfl", ctypes.c_double), ("tmax", ctypes.c_double), ("ntmax", ctypes.c_int64),
                ("precision", ctypes.c_double), ("max_its", ctypes.c_int64), ("restart", ctypes.c_int64),
                ("pc", ctypes.c_int), ("bc", ctypes.c_int), ("pc_side", ctypes.c_int), ("on_device", ctypes.c_int),
                ("dim", ctypes.c_int), ("profile", ctypes.c_int), ("fuse", ctypes.c_int)]


class WaveResult(ctypes.Structure):
    """cfp_wave_result (include/wave_system.h)."""
    _fields_ = [("steps", ctypes.c_int64), ("dt", ctypes.c_double), ("time", ctypes.c_double),
                ("total_its", ctypes.c_int64), ("max_step_its", ctypes.c_int64), ("min_step_its", ctypes.c_int64),
                ("last_reason", ctypes.c_int), ("all_converged", ctypes.c_int), ("last_residual", ctypes.c_double),
                ("last_norm_dU", ctypes.c_double), ("solve_seconds", ctypes.c_double),
                ("pc_seconds", ctypes.c_double), ("pc_calls", ctypes.c_int64), ("setup_seconds", ctypes.c_double),
                ("kappa", ctypes.c_double * 3), ("rstart", ctypes.c_int64), ("nlocal", ctypes.c_int64),
                ("loop_seconds", ctypes.c_double), ("dev_ms_", ctypes.c_double * 4),
                ("dev_launches_", ctypes.c_int64 * 4), ("fused_dots", ctypes.c_int64), ("fused_norms", ctypes.c_int64)]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "kappa" and not k.endswith("_")}
        d["kappa"] = list(self.kappa)
        d["dev_ms"] = dict(zip(("pcapply", "matmult", "vector", "copy"), self.dev_ms_))
        d["dev_launches"] = dict(zip(("pcapply", "matmult", "vector", "copy"), self.dev_launches_))
        return d


def declare(L) -> None:
    i64, dp, vp, c_int = ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int
    S, P, cs = PetscScalar, ctypes.POINTER, ctypes.c_char_p
    sig = {
        # slab-distributed plan over RCCL + single-process group
        "cfp_dist_get_unique_id": ([ctypes.c_char_p], c_int),
        "cfp_dist_unique_id_bytes": ([], c_int),
        "cfp_slab_layout": ([i64, i64, i64, c_int, c_int, P(i64)], c_int),
        "cfp_slab_work_size": ([i64, i64, i64, c_int, c_int, P(i64)], c_int),
        "cfp_slab_num_steps": ([i64, i64, i64, c_int, c_int, P(c_int)], c_int),
        "cfp_slab_step_info": ([i64, i64, i64, c_int, c_int, c_int, P(i64), P(ctypes.c_double)], c_int),
        "cfp_dist_plan_create": ([P(vp), i64, i64, i64, c_int, c_int, ctypes.c_char_p, c_int], c_int),
        "cfp_dist_plan_create_timeout": ([P(vp), i64, i64, i64, c_int, c_int, ctypes.c_char_p, c_int,
                                          ctypes.c_double], c_int),
        "cfp_dist_plan_rccl_info": ([vp, P(c_int), P(c_int), P(c_int), P(ctypes.c_double), ctypes.c_char_p, c_int],
                                    c_int),
        "cfp_rccl_version": ([P(c_int), ctypes.c_char_p, c_int], c_int),
        "cfp_rccl_blocking": ([P(c_int)], c_int),
        "cfp_dist_plan_destroy": ([vp], c_int),
        "cfp_dist_plan_create_external": ([P(vp), i64, i64, i64, c_int, c_int, c_int], c_int),
        "cfp_dist_plan_work_buffer": ([vp, P(ctypes.c_void_p)], c_int),
        "cfp_dist_plan_run_segment": ([vp, c_int, dp, dp, vp], c_int),
        "cfp_dist_plan_set_work_buffer": ([vp, dp], c_int),
        "cfp_dist_plan_set_symbol_transport": ([vp, dp], c_int),
        "cfp_dist_plan_apply": ([vp, dp, dp, vp], c_int),
        "cfp_dist_plan_profile_begin": ([vp, c_int, c_int], c_int),
        "cfp_dist_plan_profile_end": ([vp, dp, P(c_int)], c_int),
        "cfp_dist_plan_local_size": ([vp, P(i64)], c_int),
        "cfp_dist_plan_time_phases": ([vp, dp, dp, c_int, dp, vp], c_int),
        "cfp_dist_plan_num_phases": ([vp, P(c_int)], c_int),
        "cfp_dist_plan_phase_info": ([vp, c_int, P(c_int), P(c_int), P(c_int), P(c_int)], c_int),
        "cfp_group_create": ([P(vp), i64, i64, i64, c_int, P(c_int)], c_int),
        "cfp_group_destroy": ([vp], c_int),
        "cfp_group_set_symbol_transport": ([vp, dp], c_int),
        "cfp_group_apply": ([vp, P(vp), P(vp)], c_int),
        "cfp_group_set_schedule": ([vp, c_int], c_int),
        "cfp_dist_plan_set_schedule": ([vp, c_int], c_int),
        "cfp_slab_steps_count": ([i64, i64, i64, c_int, c_int, c_int, c_int, c_int, P(c_int)], c_int),
        "cfp_slab_steps_get": ([i64, i64, i64, c_int, c_int, c_int, c_int, c_int, c_int, P(i64),
                                P(ctypes.c_double)], c_int),
        "cfp_dist_plan_create_with_comm": ([P(vp), i64, i64, i64, c_int, c_int, vp, c_int], c_int),
        "cfp_dist_plan_set_exchange": ([vp, vp, vp], c_int),
        "cfp_dist_plan_set_work_buffers": ([vp, dp, dp], c_int),
        "cfp_dist_plan_num_steps": ([vp, P(c_int)], c_int),
        "cfp_dist_plan_step": ([vp, c_int, P(i64)], c_int),
        "cfp_dist_plan_run_step": ([vp, c_int, dp, dp, vp], c_int),
        "cfp_dist_plan_set_diag": ([vp, dp, vp], c_int),
        "cfp_dist_plan_clear_diag": ([vp], c_int),
        "cfp_dist_plan_forward": ([vp, dp, dp, vp], c_int),
        "cfp_dist_plan_backward": ([vp, dp, dp, vp], c_int),
        "cfp_dist_plan_set_pieces": ([vp, c_int], c_int),
        "cfp_dist_plan_pieces": ([vp, P(c_int)], c_int),
        "cfp_group_set_pieces": ([vp, c_int], c_int),
        "cfp_dist_plan_use_diag": ([vp, c_int], c_int),
        # PETSc stand-in: communicators and distributed objects
        "MPI_Comm_size": ([c_int, P(c_int)], c_int),
        "MPI_Comm_rank": ([c_int, P(c_int)], c_int),
        "PetscMiniCommCreate": ([c_int, c_int, vp, P(c_int)], c_int),
        "PetscMiniCommCreateRCCL": ([c_int, c_int, ctypes.c_char_p, P(c_int)], c_int),
        "PetscMiniCommDestroy": ([P(c_int)], c_int),
        "PetscMiniSetCommWorld": ([c_int], c_int),
        "PetscMiniCommResolve": ([c_int, P(c_int)], c_int),
        "PetscMiniAllreduce": ([c_int, P(ctypes.c_double), i64, c_int], c_int),
        "PetscMiniCommGetNCCL": ([c_int, P(vp)], c_int),
        "PetscMiniMatAIJGetFormat": ([vp, P(c_int)], c_int),
        "VecCreateMPI": ([c_int, i64, i64, P(vp)], c_int),
        "VecCreateMPIHIP": ([c_int, i64, i64, P(vp)], c_int),
        "VecCreateMPIHIPWithArray": ([c_int, i64, i64, i64, vp, P(vp)], c_int),
        "VecGetComm": ([vp, P(c_int)], c_int),
        "VecGetLocalSize": ([vp, P(i64)], c_int),
        "VecGetOwnershipRange": ([vp, P(i64), P(i64)], c_int),
        "MatGetLocalSize": ([vp, P(i64), P(i64)], c_int),
        "MatGetComm": ([vp, P(c_int)], c_int),
        "MatFFTHIPGetDistPlan": ([vp, P(vp)], c_int),
        # PETSc stand-in
        "PetscErrorLastMessage": ([], cs),
        "VecMiniSetStream": ([vp], c_int),
        "VecCreateSeq": ([c_int, i64, P(vp)], c_int),
        "VecCreateSeqHIP": ([c_int, i64, P(vp)], c_int),
        "VecCreateSeqHIPWithArray": ([c_int, i64, i64, vp, P(vp)], c_int),
        "VecDuplicate": ([vp, P(vp)], c_int),
        "VecDestroy": ([P(vp)], c_int),
        "VecGetSize": ([vp, P(i64)], c_int),
        "VecGetArray": ([vp, P(vp)], c_int),
        "VecRestoreArray": ([vp, P(vp)], c_int),
        "VecGetArrayRead": ([vp, P(vp)], c_int),
        "VecRestoreArrayRead": ([vp, P(vp)], c_int),
        "VecHIPGetArray": ([vp, P(vp)], c_int),
        "VecHIPRestoreArray": ([vp, P(vp)], c_int),
        "VecSet": ([vp, S], c_int),
        "VecSetValue": ([vp, i64, S, c_int], c_int),
        "VecAssemblyBegin": ([vp], c_int),
        "VecAssemblyEnd": ([vp], c_int),
        "VecCopy": ([vp, vp], c_int),
        "VecScale": ([vp, S], c_int),
        "VecShift": ([vp, S], c_int),
        "VecAXPY": ([vp, S, vp], c_int),
        "VecAYPX": ([vp, S, vp], c_int),
        "VecWAXPY": ([vp, S, vp, vp], c_int),
        "VecPointwiseDivide": ([vp, vp, vp], c_int),
        "VecPointwiseMult": ([vp, vp, vp], c_int),
        "VecDot": ([vp, vp, P(S)], c_int),
        "VecNorm": ([vp, c_int, P(ctypes.c_double)], c_int),
        "MatCreateSeqAIJWithArrays": ([c_int, i64, i64, P(i64), P(i64), vp, P(vp)], c_int),
        "MatCreateFFT": ([c_int, i64, P(i64), cs, P(vp)], c_int),
        "MatCreateFFTHIP": ([c_int, i64, P(i64), P(vp)], c_int),
        "MatFFTHIPGetPlan": ([vp, P(vp)], c_int),
        "MatFFTHIPGetSolveCounts": ([vp, P(i64), P(i64)], c_int),
        "PetscObjectStateGet": ([vp, P(i64)], c_int),
        "PetscObjectGetId": ([vp, P(i64)], c_int),
        "MatCreateVecsFFTW": ([vp, P(vp), P(vp), P(vp)], c_int),
        "MatGetSize": ([vp, P(i64), P(i64)], c_int),
        "MatCreateAIJ": ([c_int, i64, i64, i64, i64, i64, vp, i64, vp, P(vp)], c_int),
        "MatSetValues": ([vp, i64, P(i64), i64, P(i64), vp, c_int], c_int),
        "MatAssemblyBegin": ([vp, c_int], c_int),
        "MatAssemblyEnd": ([vp, c_int], c_int),
        "MatGetOwnershipRange": ([vp, P(i64), P(i64)], c_int),
        "PetscMiniMatMPIAIJGetHalo": ([vp, P(i64), P(i64)], c_int),
        "MatMult": ([vp, vp, vp], c_int),
        "MatMultTranspose": ([vp, vp, vp], c_int),
        "MatShift": ([vp, S], c_int),
        "MatDestroy": ([P(vp)], c_int),
        "PCCreate": ([c_int, P(vp)], c_int),
        "PCSetType": ([vp, cs], c_int),
        "PCShellSetContext": ([vp, vp], c_int),
        "PCShellGetContext": ([vp, P(vp)], c_int),
        "PCShellSetApply": ([vp, vp], c_int),
        "PCShellSetSetUp": ([vp, vp], c_int),
        "PCShellSetDestroy": ([vp, vp], c_int),
        "PCSetUp": ([vp], c_int),
        "PCApply": ([vp, vp, vp], c_int),
        "PCDestroy": ([P(vp)], c_int),
        "VecMDot": ([vp, i64, P(vp), P(S)], c_int),
        "VecMAXPY": ([vp, i64, P(S), P(vp)], c_int),
        "KSPCreate": ([c_int, P(vp)], c_int),
        "KSPSetType": ([vp, cs], c_int),
        "KSPSetTolerances": ([vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, i64], c_int),
        "KSPGMRESSetRestart": ([vp, i64], c_int),
        "KSPSetPCSide": ([vp, c_int], c_int),
        "KSPSetInitialGuessNonzero": ([vp, c_int], c_int),
        "KSPGetPC": ([vp, P(vp)], c_int),
        "KSPSetOperators": ([vp, vp, vp], c_int),
        "KSPSetUp": ([vp], c_int),
        "KSPSolve": ([vp, vp, vp], c_int),
        "KSPGetConvergedReason": ([vp, P(c_int)], c_int),
        "KSPGetIterationNumber": ([vp, P(i64)], c_int),
        "KSPGetResidualNorm": ([vp, P(ctypes.c_double)], c_int),
        "KSPMiniGetPCApplyStats": ([vp, P(i64), P(ctypes.c_double)], c_int),
        "KSPMiniSetUpWork": ([vp, vp], c_int),
        "KSPDestroy": ([P(vp)], c_int),
        # transport operator + GMRES time loop (include/transport_equation.h)
        "cfp_transport_csr": ([i64, i64, i64, P(ctypes.c_double), ctypes.c_double, P(ctypes.c_double), c_int,
                               ctypes.c_double, P(i64), P(i64), P(ctypes.c_double), P(i64)], c_int),
        "cfp_cartesian_min_ratio_vol_surf": ([c_int, P(ctypes.c_double)], ctypes.c_double),
        "computeDivergenceMatrixCartesian": ([i64, i64, i64, P(ctypes.c_double), ctypes.c_double,
                                              P(ctypes.c_double), i64, P(vp)], c_int),
        "initial_conditions_shock_cartesian": ([i64, i64, i64, P(ctypes.c_double), P(ctypes.c_double), vp], c_int),
        "cfp_transport_config_default": ([P(TransportConfig), i64], None),
        "TransportEquationGMRES": ([P(TransportConfig), P(TransportResult), P(ctypes.c_double)], c_int),
        "TransportEquationFFTDirect": ([P(TransportConfig), P(TransportResult), P(ctypes.c_double)], c_int),
        # unstructured meshes, the PCSHELL remap and the mesh transport loop (include/mesh_unstructured.h)
        "cfp_mesh_read_gmsh": ([cs, P(vp)], c_int),
        "cfp_mesh_create": ([i64, P(ctypes.c_double), i64, P(i64), P(i64), P(vp)], c_int),
        "cfp_mesh_destroy": ([vp], c_int),
        "cfp_mesh_info": ([vp, P(i64), P(i64), P(i64), P(ctypes.c_double)], c_int),
        "cfp_mesh_cell_geometry": ([vp, P(ctypes.c_double), P(ctypes.c_double)], c_int),
        "cfp_mesh_min_ratio_vol_surf": ([vp, P(ctypes.c_double)], c_int),
        "cfp_mesh_faces": ([vp, P(i64), P(i64), P(ctypes.c_double), P(ctypes.c_double)], c_int),
        "cfp_mesh_crude_matrix_cartesian": ([vp, i64, i64, i64, P(ctypes.c_double), P(i64), P(i64), P(i64),
                                             P(ctypes.c_double)], c_int),
        "cfp_mesh_transport_csr": ([vp, ctypes.c_double, P(ctypes.c_double), c_int, ctypes.c_double, P(i64), P(i64),
                                    P(i64), P(ctypes.c_double)], c_int),
        "MatCreateMeshCartesianRemap": ([vp, i64, i64, i64, P(ctypes.c_double), P(vp), P(vp)], c_int),
        "getFFTPrec3DContextMesh": ([i64, S, S, S, S, vp, vp], c_int),
        "FFTPrec3DContextDestroyRemap": ([vp], c_int),
        "initial_conditions_shock_mesh": ([vp, vp], c_int),
        "TransportEquationGMRESMesh": ([vp, P(TransportConfig), P(TransportResult), P(ctypes.c_double)], c_int),
        # wave system (include/wave_system.h)
        "cfp_wave_plan_create": ([P(vp), i64, i64, i64, c_int], c_int),
        "cfp_wave_plan_create_dim": ([P(vp), i64, i64, i64, c_int, c_int], c_int),
        "cfp_wave_plan_destroy": ([vp], c_int),
        "cfp_wave_plan_set_symbol": ([vp, P(ctypes.c_double), ctypes.c_double], c_int),
        "cfp_wave_plan_apply": ([vp, dp, dp, vp], c_int),
        "cfp_wave_plan_apply_dots": ([vp, dp, dp, vp, c_int, ctypes.POINTER(ctypes.c_void_p), dp, P(c_int)], c_int),
        "cfp_wave_plan_set_schedule": ([vp, c_int], c_int),
        "cfp_wave_plan_forward": ([vp, dp, dp, vp], c_int),
        "cfp_wave_plan_backward": ([vp, dp, dp, vp], c_int),
        "cfp_wave_plan_num_passes": ([vp, P(c_int)], c_int),
        "cfp_wave_plan_time_passes": ([vp, dp, dp, c_int, dp, vp], c_int),
        "cfp_wave_csr": ([i64, i64, i64, P(ctypes.c_double), ctypes.c_double, ctypes.c_double, c_int,
                          ctypes.c_double, P(i64), P(i64), P(ctypes.c_double), P(i64)], c_int),
        "cfp_wave_csr_dim": ([i64, i64, i64, c_int, P(ctypes.c_double), ctypes.c_double, ctypes.c_double, c_int,
                              ctypes.c_double, P(i64), P(i64), P(ctypes.c_double), P(i64)], c_int),
        "computeDivergenceMatrixWaveCartesian": ([i64, i64, i64, P(ctypes.c_double), ctypes.c_double,
                                                  ctypes.c_double, i64, P(vp)], c_int),
        "computeDivergenceMatrixWaveCartesianDim": ([i64, i64, i64, i64, P(ctypes.c_double), ctypes.c_double,
                                                     ctypes.c_double, i64, P(vp)], c_int),
        "initial_conditions_shock_wave": ([i64, i64, i64, P(ctypes.c_double), P(ctypes.c_double), vp], c_int),
        "applyFFT3DPrecWave": ([vp, vp, vp], c_int),
        "setupFFTPrec3DWave": ([vp], c_int),
        "destroyFFTPrec3DWave": ([vp], c_int),
        "cfp_wave_config_default": ([P(WaveConfig), i64], None),
        "cfp_wave_config_default_dim": ([P(WaveConfig), i64, c_int], None),
        "WaveSystemGMRES": ([P(WaveConfig), P(WaveResult), P(ctypes.c_double)], c_int),
        # the reference-named boundary
        "applyFFT3DPrecTransport": ([vp, vp, vp], c_int),
        "setupFFTPrec3D": ([vp], c_int),
        "destroyFFTPrec3D": ([vp], c_int),
        "getFFTPrec3DContext": ([i64, S, i64, S, S, S, S, S, S, S, S, S, P(FFTPrecTransportContext)], c_int),
        "FFTPrecTransportContextCreate": ([P(vp)], c_int),
        "FFTPrecTransportContextSetRemapBack": ([P(FFTPrecTransportContext), vp], c_int),
        "FFTPrecTransportContextGetRemapBack": ([P(FFTPrecTransportContext), P(vp)], c_int),
        "FFTPrecTransportContextDestroy": ([P(vp)], c_int),
        "solve_3D": ([vp, vp, vp, vp, vp, i64], c_int),
        "build_transport_col": ([vp, i64], c_int),
        "build_diag_mat_vec_3D": ([vp, vp, vp, vp, i64, i64, i64, S, S, S], c_int),
        "FftTransportSolver": ([i64, i64, i64, S, S, S, vp, vp, vp], c_int),
        "Fft3DTransportSolver": ([i64, i64, i64, S, S, S, S, S, S, S, vp, vp, vp], c_int),
        "Fft2DTransportSolver": ([i64, i64, S, S, S, S, S, vp, vp, vp], c_int),
        "Fft1DTransportSolver": ([i64, S, S, S, vp, vp, vp], c_int),
        "PetscFft3DTransportSolver": ([StructuredTransportContext, vp, vp], c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
