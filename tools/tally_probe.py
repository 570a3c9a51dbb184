#!/usr/bin/env python3
"""cfg4 tally (1M rows, C=4) warm and cold per workgroup chunk count
(the block_chunks test hook, read at snapshot upload): back-to-back HIP-event rate and
the median of single launches after a 512 MiB scrub. Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    p = synth.config4()
    eng = Engine(0)
    stream = torch.cuda.current_stream().cuda_stream
    C, L = len(p.classes), p.topology.n_leaves
    cap = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
    scrub = torch.zeros(128 << 20, dtype=torch.int32, device="cuda")
    tb = bench.tally_bytes(p)
    for ch in (1, 2, 3, 4):
        os.environ["JSP_TEST_HOOKS"] = f"block_chunks={ch}"
        eng.load(p)
        fn = lambda: eng.tally_device(cap.data_ptr(), cap[-1].data_ptr(), L, stream)  # noqa: E731
        for _ in range(10):
            fn()
        warm = bench.event_loop_us(fn, 200, stream)
        cold = bench.cold_us(fn, 20, stream, scrub)
        eng.check()
        print(f"chunks {ch}: warm {warm:.2f} us ({tb / warm / 1e3:.0f} GB/s), cold {cold:.2f} us "
              f"({tb / cold / 1e3:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
