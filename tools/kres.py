#!/usr/bin/env python3
"""Register use of the gfx950 kernels in a built library (CPU only):
python tools/kres.py [LIB] [NAME-FILTER]. VGPRs, SGPRs, spills, scratch, LDS."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_kernel_resources as T  # noqa: E402


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else T.LIB
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    T.LIB = lib
    for name, k in sorted(T._kernel_notes().items()):
        if flt in name:
            print(f"{name[:90]:90s} vgpr={k.get('.vgpr_count')} agpr={k.get('.agpr_count')} sgpr={k.get('.sgpr_count')} "
                  f"vspill={k.get('.vgpr_spill_count')} sspill={k.get('.sgpr_spill_count')} "
                  f"scratch={k.get('.private_segment_fixed_size')} lds={k.get('.group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
