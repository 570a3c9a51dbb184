#!/usr/bin/env python3
"""Write the gfx950 code object of a built library to a file (CPU only), for
llvm-objdump: python tools/dump_co.py [LIB] OUT.co"""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_kernel_resources as T  # noqa: E402


def main():
    lib = sys.argv[1] if len(sys.argv) > 2 else T.LIB
    out = sys.argv[-1]
    blob = open(lib, "rb").read()
    fat = next(data for name, _, data in T._elf_sections(blob) if name == ".hip_fatbin")
    n, = struct.unpack_from("<Q", fat, 24)
    pos = 32
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", fat, pos)
        triple = fat[pos + 24:pos + 24 + tlen].decode()
        pos += 24 + tlen
        if triple.endswith("gfx950"):
            open(out, "wb").write(fat[off:off + size])
            return


if __name__ == "__main__":
    main()
