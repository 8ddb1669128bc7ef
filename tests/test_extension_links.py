"""The in-tree HIP extension must load (every exported launcher resolved) even on a CPU-only
host: an unresolved symbol would otherwise only surface on the GPU box."""
import glob
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["_dtf_hip", "_dtf_native"])
def test_extension_imports(name):
    if not glob.glob(os.path.join(ROOT, "distributedtensorflow_amd", "_lib", name + "*.so")):
        pytest.skip(f"{name} not built")
    import importlib
    mod = importlib.import_module(f"distributedtensorflow_amd._lib.{name}")
    assert mod is not None
