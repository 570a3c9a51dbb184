#!/bin/bash
# round-4 evidence pass: GPU tests, service stamps, bench (driver flags)
out=gpurun_out/r4/${1:-p2}
mkdir -p $out
timeout -k 10 120 ./tools/bin/block_probe 15 > $out/block_probe.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 120 python tools/dbg_clk.py > $out/svc_stamps.txt 2>&1 && JSP_LIB_PATH=tools/bin/ab_clk/libjsplace.so timeout -k 10 120 python tools/dbg_clk.py >> $out/svc_stamps.txt 2>&1 || exit 3
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit 4
