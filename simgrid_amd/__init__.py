"""simgrid_amd — MI355X-native linear max-min (LMM) solver for SimGrid's resource-sharing core.

The product is liblmm_amd.so (HIP kernels for gfx950 + host lmm::System + C ABI, see
include/lmm/*.h).  simgrid_amd.lmm is its Python mirror of the reference lmm::System API.
"""
from . import lmm  # noqa: F401
