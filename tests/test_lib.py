"""libqknit.so builds for gfx950, loads, and exports every symbol include/qknit.h declares."""
import os
import re

from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import _lib
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.build import HEADER, build_library


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(qk_\w+)\s*\(", src, re.M)))


def test_library_builds_and_exports_header_symbols():
    path = build_library()
    assert os.path.exists(path)
    lib = _lib.lib()
    decl = declared_functions()
    assert len(decl) >= 11
    for name in decl:
        assert hasattr(lib, name), name
    assert set(decl) == set(_lib.SIGNATURES), "ctypes signatures out of sync with qknit.h"
    assert b"gfx950" in lib.qk_version()


def test_struct_layouts_match_header():
    import ctypes

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import sweep_plan

    assert sweep_plan.OP_DTYPE.itemsize == 32
    assert sweep_plan.GROUP_DTYPE.itemsize == 32
    assert ctypes.sizeof(_lib.QkPass) == 24 == sweep_plan.PASS_DTYPE.itemsize
    assert ctypes.sizeof(_lib.QkProgram) == 6 * 4 + 4 * 8


def test_no_compute_without_device():
    # argument validation runs host-side and reports through qk_last_error
    import ctypes

    lib = _lib.lib()
    assert lib.qk_ctx_create(0, None) != 0
    assert lib.qk_sweep(None, None, 0, None, None, None, 0, None) != 0
    assert lib.qk_last_error(None) == b"null context"


def test_new_entry_points_validate_arguments_without_device():
    """Sampling and fused-sweep entry points reject a null context before touching the GPU."""
    lib = _lib.lib()
    assert lib.qk_sample_cdf(None, 1, None, 4, None, None) != 0
    assert lib.qk_sample_counts(None, 1, 0, None, None, None, 4, None, 10, 0, None) != 0
    assert lib.qk_fold_counts(None, 1, None, 4, None, None, 10, 0.0, None) != 0
    assert lib.qk_sweep_compiled_labels(None, None, None, 1, None, None, 1, None, None, 0, None) != 0
