#!/bin/bash
# round-4: service A/B stamps, service GPU tests, bench
out=gpurun_out/r4/${1:-p4}
mkdir -p $out
timeout -k 10 120 ./tools/bin/block_probe 15 > $out/block_probe.txt 2>&1 || exit 1
timeout -k 10 100 python tools/cold_probe2.py 30 > $out/cold_probe2.txt 2>&1 && JSP_SVC_WAKE=0 timeout -k 10 100 python tools/cold_probe2.py 30 >> $out/cold_probe2.txt 2>&1 && true || exit 3
timeout -k 10 400 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread --durations=10 > $out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit 4
