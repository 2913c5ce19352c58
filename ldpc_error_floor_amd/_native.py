"""Loader for the in-tree native extension.  There is no CPU fallback: if the HIP
extension is missing the product path raises instead of silently computing elsewhere."""
from __future__ import annotations

import ctypes
import importlib
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libldpc_nms.so")
_mod = None


class NativeExtensionMissing(RuntimeError):
    pass


def load():
    """Import ``_ldpc_nms`` (pybind11) — torch is imported first so that the process uses
    torch's HIP runtime (same SONAME as /opt/rocm's)."""
    global _mod
    if _mod is not None:
        return _mod
    import torch  # noqa: F401  (HIP runtime first)
    try:
        _mod = importlib.import_module("ldpc_error_floor_amd._ldpc_nms")
    except ImportError as e:
        raise NativeExtensionMissing(
            "ldpc_error_floor_amd HIP extension is not built "
            "(run `python -m ldpc_error_floor_amd.build` or __graft_entry__.build()): " + str(e))
    return _mod


def load_cabi() -> ctypes.CDLL:
    """The raw C-ABI library (for ABI checks and non-Python hosts)."""
    if not os.path.exists(LIB_PATH):
        raise NativeExtensionMissing(f"{LIB_PATH} not built")
    return ctypes.CDLL(LIB_PATH)
