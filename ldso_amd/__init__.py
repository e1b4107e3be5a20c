"""ldso_amd -- MI355X-native LDSO photometric bundle-adjustment hot path.

The product is the HIP/C++ library ``ldso_amd/lib/libldso_ba.so`` behind the C ABI in
``include/ldso_ba.h``.  This package is a thin Python face of that ABI (used by tests and
bench.py); it performs no numerical work itself.
"""
from . import _lib
from ._lib import FLAG_ACTIVE, FLAG_NEW, RES_IN, RES_OOB, RES_OUTLIER
from .context import BAContext
from .window import Window

__all__ = ["BAContext", "Window", "RES_IN", "RES_OOB", "RES_OUTLIER", "FLAG_ACTIVE", "FLAG_NEW", "lib"]


def lib():
    return _lib.lib()
