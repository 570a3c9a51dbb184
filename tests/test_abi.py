"""CPU tests of the C-ABI boundary: the in-tree library loads, exports every
entry point include/jsplace.h declares with the declared structs' layout, and
fails loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re

import pytest

from jobset_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "jsplace.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(jsp_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "jsp_place" in names and "jsp_engine_create" in names and len(names) >= 18


def test_library_exports_every_declared_symbol():
    lib = native.lib()
    for name in declared_functions():
        assert hasattr(lib, name), f"libjsplace.so does not export {name}"
    bound = {n for n, _, _ in native.SIGNATURES}
    assert bound == set(declared_functions()), "native.SIGNATURES out of sync with include/jsplace.h"


def test_abi_version_and_struct_layout():
    lib = native.lib()
    assert lib.jsp_abi_version() == 6
    # layouts the Go cgo wrapper relies on
    assert ctypes.sizeof(native.JspJobClass) == 8 * 4 * 2 + 4 * 3 + 4 * 4 + 4  # 100 B + 4 pad
    assert ctypes.sizeof(native.JspTopology) == 4 + 4 * 4 + 4 + 8 * 4
    assert ctypes.sizeof(native.JspStats) == 24


def test_library_reads_only_operational_switches():
    """The shipped library names no A/B switch: the only environment
    variables it reads are the operational ones and the tests' hook string
    (jsplace.h "Environment")."""
    blob = open(os.path.join(ROOT, "jobset_amd", "libjsplace.so"), "rb").read()
    names = {n.decode() for n in re.findall(rb"JSP_[A-Z0-9_]+", blob)}
    assert names <= {"JSP_SERVICE", "JSP_SERVICE_IDLE_MS", "JSP_RCCL_LIB", "JSP_TEST_HOOKS"}, names


def test_no_gpu_fails_loudly():
    if native.device_count() > 0:
        pytest.skip("a GPU is present")
    from jobset_amd.engine import Engine
    with pytest.raises(native.JspError) as ei:
        Engine(0)
    assert ei.value.code == native.JSP_EHIP
    assert "no HIP device" in str(ei.value)


def test_null_engine_is_einval():
    lib = native.lib()
    assert lib.jsp_engine_sync(None) == native.JSP_EINVAL
    assert b"NULL" in lib.jsp_last_error()


def test_device_set_without_gpu_fails_loudly():
    if native.device_count() > 0:
        pytest.skip("a GPU is present")
    from jobset_amd.engine import Engine
    with pytest.raises(native.JspError) as ei:
        Engine(devices=[0, 0])
    assert ei.value.code == native.JSP_EHIP
    with pytest.raises(native.JspError) as ei:
        Engine(devices=[])
    assert ei.value.code == native.JSP_EINVAL
