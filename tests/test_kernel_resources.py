"""Code-generation guard for the built gfx950 kernels (CPU only, no GPU).

Reads the kernel descriptors of the gfx950 code object inside
jobset_amd/libjsplace.so and checks that no kernel uses scratch: no private
segment, no VGPR spills, no dynamic stack. A modified copy of a kernel-argument
struct whose arrays are indexed at run time, or a runtime-indexed local array,
would land in scratch ("code-generation rules").
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "jobset_amd", "libjsplace.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernel_notes(tmp_path):
    bundler = os.path.join(LLVM, "clang-offload-bundler")
    readelf = os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(LIB) and shutil.which("objcopy") and os.path.exists(bundler)
            and os.path.exists(readelf)):
        pytest.skip("library or ROCm LLVM tools absent")
    fat = tmp_path / "fatbin.bin"
    co = tmp_path / "gfx950.co"
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", LIB], check=True)
    subprocess.run([bundler, "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                    f"--output={co}", "--unbundle"], check=True)
    notes = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    kernels = {}
    cur = None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|uses_dynamic_stack):\s+(\S+)", line)
        if m and cur is not None:
            kernels[cur][m.group(1)] = m.group(2)
    return kernels


def test_no_kernel_uses_scratch(tmp_path):
    kernels = _kernel_notes(tmp_path)
    # every kernel family of the engine is in the library
    for fam in ("tally_kernel", "feas_kernel", "assign_kernel", "expand_kernel", "place_compact_kernel",
                "place_fused_kernel", "place_service_kernel", "place_fused_service_kernel"):
        assert any(fam in k for k in kernels), fam
    bad = {k: v for k, v in kernels.items()
           if v.get("private_segment_fixed_size") != "0" or v.get("vgpr_spill_count") != "0"
           or v.get("uses_dynamic_stack") != "false"}
    assert not bad, bad
