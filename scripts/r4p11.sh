#!/bin/bash
# inline patches: service phases with patched rows, cold/warm probe, full GPU suite, bench
out=gpurun_out/r4/${1:-p13}
mkdir -p $out
timeout -k 10 200 python tools/svc_probe.py 500 > $out/svc_probe.txt 2>&1 || exit 5
timeout -k 10 150 python tools/cold_probe2.py 30 > $out/cold_probe2.txt 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=10 > $out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit 4
