"""The C-ABI library loads and exports every entry point include/kbgpu.h declares (no GPU needed)."""
import ctypes
import os
import re

from scheduler_amd import runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "kbgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kb_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = runtime.load_library()
    decl = declared_functions()
    assert "kb_place_job" in decl and "kb_allocate" in decl
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(runtime.EXPORTS) == decl


def test_abi_version():
    assert runtime.load_library().kb_abi_version() == runtime.ABI_VERSION == 2


def test_struct_layouts_match_header():
    # sizes follow the C layout of include/kbgpu.h (x86-64 SysV, natural alignment)
    assert ctypes.sizeof(runtime.kb_nodes) == 16 + 18 * 8
    assert ctypes.sizeof(runtime.kb_job_result) == 16 + 16 * 4
    assert ctypes.sizeof(runtime.kb_config) == 9 * 4
    from scheduler_amd import export
    assert export.SPEC_DTYPE.itemsize == 112


def test_no_device_fails_loudly():
    # In this container there is no GPU: the product must refuse, never fall back to the CPU.
    import pytest
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    with pytest.raises(runtime.KbError):
        runtime.Context(0)
