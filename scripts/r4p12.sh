#!/bin/bash
# waker thread: cold probe (host vs GPU), service tests, full GPU suite, bench
out=gpurun_out/r4/${1:-p17}
mkdir -p $out
timeout -k 10 200 python tools/cold_probe3.py 20 > $out/cold_probe3.txt 2>&1 || exit 3
timeout -k 10 300 python -u -m pytest tests/test_service_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_svc.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=10 > $out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit 4
