"""The C-ABI library loads and exports every entry point include/kbgpu.h declares (no GPU needed)."""
import ctypes
import os
import re

from scheduler_amd import runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "kbgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kb_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = runtime.load_library()
    decl = declared_functions()
    assert "kb_place_job" in decl and "kb_allocate" in decl
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(runtime.EXPORTS) == decl


def test_abi_version():
    assert runtime.load_library().kb_abi_version() == runtime.ABI_VERSION == 16


def test_struct_layouts_match_header():
    # sizes follow the C layout of include/kbgpu.h (x86-64 SysV, natural alignment)
    assert ctypes.sizeof(runtime.kb_nodes) == 16 + 18 * 8
    assert ctypes.sizeof(runtime.kb_job_result) == 16 + 17 * 4
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


def test_struct_sizes_agree_with_the_c_compiler(tmp_path):
    """Every ABI struct: gcc's sizeof(include/kbgpu.h) == the ctypes / numpy layout the binding uses."""
    import subprocess
    from scheduler_amd import affinity as A
    from scheduler_amd import export
    ours = {"kb_nodes": ctypes.sizeof(runtime.kb_nodes), "kb_specs": ctypes.sizeof(runtime.kb_specs),
            "kb_config": ctypes.sizeof(runtime.kb_config), "kb_opts": ctypes.sizeof(runtime.kb_opts),
            "kb_job_req": ctypes.sizeof(runtime.kb_job_req), "kb_job_result": ctypes.sizeof(runtime.kb_job_result),
            "kb_stats": ctypes.sizeof(runtime.kb_stats), "kb_affinity": ctypes.sizeof(runtime.kb_affinity),
            "kb_shard": ctypes.sizeof(runtime.kb_shard),
            "kb_session": ctypes.sizeof(runtime.kb_session), "kb_cycle_result": ctypes.sizeof(runtime.kb_cycle_result),
            "kb_spec": export.SPEC_DTYPE.itemsize, "kb_req": export.REQ_DTYPE.itemsize,
            "kb_term": export.TERM_DTYPE.itemsize, "kb_port": export.PORT_DTYPE.itemsize,
            "kb_aff_table": A.AFF_TABLE_DTYPE.itemsize, "kb_aff_check": A.AFF_CHECK_DTYPE.itemsize,
            "kb_ipa_hist": A.IPA_HIST_DTYPE.itemsize, "kb_ipa_incr": A.IPA_INCR_DTYPE.itemsize,
            "kb_aff_spec": A.AFF_SPEC_DTYPE.itemsize, "kb_row_delta": runtime.ROW_DELTA_DTYPE.itemsize}
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "kbgpu.h"\nint main(void) {\n' +
                   "".join(f'  printf("{k} %zu\\n", sizeof({k}));\n' for k in ours) + "  return 0;\n}\n")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                           text=True).stdout.splitlines())
    assert {k: int(v) for k, v in got.items()} == ours
