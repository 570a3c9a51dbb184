#!/bin/bash
out=gpurun_out/r4/${1:-p27}
mkdir -p $out
timeout -k 10 120 python tools/stop_probe.py > $out/stop_spin.txt 2>&1 || exit 3
JSP_SVC_STOP_SPIN=0 timeout -k 10 120 python tools/stop_probe.py > $out/stop_block.txt 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 4
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench.err || exit 6
