"""MI355X-native (gfx950) differential attention.

Drop-in module mirrors of the reference (``diff_transformer``,
``Ndiff_transformer``, ``control``), the fused HIP ops behind them (``ops``,
C ABI in ``include/diffattn.h``) and data-parallel training over RCCL
(``train``, ``dp``).
"""
from . import _lib, ops  # noqa: F401

__version__ = "0.1.0"
