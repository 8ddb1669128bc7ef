"""Loader for the host-runtime extension ``_dtf_native`` (C++17, built in-tree by ``_build``).

Builds it on first use when missing (g++ only, seconds) so CPU-only environments work without
an explicit build step.
"""
from __future__ import annotations

import importlib
import threading

_lock = threading.Lock()
_mod = None


def lib():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            try:
                _mod = importlib.import_module("distributedtensorflow_amd._lib._dtf_native")
            except ImportError:
                from .. import _build
                _build.build_native()
                importlib.invalidate_caches()
                _mod = importlib.import_module("distributedtensorflow_amd._lib._dtf_native")
    return _mod


def crc32c(data: bytes, init: int = 0) -> int:
    return lib().crc32c(data, init)


def masked_crc32c(data: bytes) -> int:
    return lib().masked_crc32c(data)
