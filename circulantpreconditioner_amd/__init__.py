"""MI355X-native circulant / block-circulant FFT preconditioner.

The product is ``lib/libcirculant_fft.so`` (hand-written HIP kernels for gfx950 +
a C ABI, ``include/*.h``).  This package is the Python host mirror of the
reference's operator interface (``src/FftLinearSolver_3D.h``,
``src/PCSHELLFft_3D.hxx``); PyTorch supplies device memory and streams only.
"""
from ._lib import CirculantError, LIB_PATH, lib  # noqa: F401
from .plan import (CirculantPlan, RealPlan, build_diag_3d, fill_uniform, pointwise_divide,  # noqa: F401
                   scale, transport_symbol_1d)

__version__ = "0.1.0"
