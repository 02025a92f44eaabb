"""odp_amd — MI355X-native ODP receive-path classifier.

The product is the C-ABI shared library ``odp_amd/lib/libodpg.so`` (HIP
kernels for gfx950 + the host runtime + the ``odp_cls_*`` object model).
This package only loads it (``odp_amd._lib``), mirrors the ODP
classification API for Python callers (``odp_amd.cls``) and generates
synthetic traffic (``odp_amd.gen``).
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
