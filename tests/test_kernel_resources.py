"""Code-generation guard for the built gfx950 kernels (CPU only, no GPU).

Reads the kernel descriptors of the gfx950 code object inside
jobset_amd/libjsplace.so and checks that no kernel uses scratch: no private
segment, no VGPR spills, no dynamic stack. A modified copy of a kernel-argument
struct whose arrays are indexed at run time, or a runtime-indexed local array,
would land in scratch ("code-generation rules").
"""
import os
import struct

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "jobset_amd", "libjsplace.so")


# Pure-Python reading (no child processes: forking after the HIP runtime is
# loaded by an earlier test has crashed the test process later).
def _elf_sections(blob):
    shoff, = struct.unpack_from("<Q", blob, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", blob, 0x3A)
    heads = [struct.unpack_from("<IIQQQQIIQQ", blob, shoff + i * shentsize) for i in range(shnum)]
    stro = heads[shstrndx][4]
    for h in heads:
        end = blob.index(b"\0", stro + h[0])
        yield blob[stro + h[0]:end].decode(), h[1], blob[h[4]:h[4] + h[5]]


def _kernel_notes():
    msgpack = pytest.importorskip("msgpack")
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    with open(LIB, "rb") as f:
        lib = f.read()
    fat = next(data for name, _, data in _elf_sections(lib) if name == ".hip_fatbin")
    assert fat[:24] == b"__CLANG_OFFLOAD_BUNDLE__", "uncompressed offload bundle expected"
    n, = struct.unpack_from("<Q", fat, 24)
    pos, co = 32, None
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", fat, pos)
        triple = fat[pos + 24:pos + 24 + tlen].decode()
        pos += 24 + tlen
        if triple.endswith("gfx950"):
            co = fat[off:off + size]
    assert co is not None, "no gfx950 code object in the library"
    for _, typ, data in _elf_sections(co):
        if typ != 7:  # SHT_NOTE
            continue
        q = 0
        while q + 12 <= len(data):
            namesz, descsz, ntype = struct.unpack_from("<III", data, q)
            name = data[q + 12:q + 12 + namesz].rstrip(b"\0")
            d0 = q + 12 + ((namesz + 3) & ~3)
            if name == b"AMDGPU" and ntype == 32:  # NT_AMDGPU_METADATA (msgpack)
                meta = msgpack.unpackb(data[d0:d0 + descsz], raw=False)
                return {k[".name"]: k for k in meta["amdhsa.kernels"]}
            q = d0 + ((descsz + 3) & ~3)
    raise AssertionError("no AMDGPU metadata note")


def test_no_kernel_uses_scratch():
    kernels = _kernel_notes()
    # every kernel family of the engine is in the library
    for fam in ("tally_kernel", "feas_kernel", "assign_kernel", "expand_kernel", "place_compact_kernel",
                "place_fused_kernel", "place_service_kernel", "place_split_service_kernel", "assign_level_kernel"):
        assert any(fam in k for k in kernels), fam
    # The resident compaction service at R = 1 runs at the SGPR limit (106):
    # the backend reserves a 36-byte frame for its SGPR spill bookkeeping that
    # its code never touches (no scratch instruction in the disassembly, and
    # no alloca in its LLVM IR). Any other size or kernel fails.
    unused_frame = {"place_service_kernelILi1ELi1E": 36, "place_service_kernelILi2ELi1E": 36}

    def frame_ok(name, v):
        size = v.get(".private_segment_fixed_size")
        return size == 0 or any(k in name and size == n for k, n in unused_frame.items())
    bad = {k: v for k, v in kernels.items()
           if not frame_ok(k, v) or v.get(".vgpr_spill_count") != 0
           or v.get(".uses_dynamic_stack") is not False}
    assert not bad, bad
