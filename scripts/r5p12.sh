#!/bin/bash
# run-based expansion: service + engine GPU tests, A/B, driver bench
out=gpurun_out/r5/${1:-p12}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -60 $out/pytest.log; exit 2; }
tail -2 $out/pytest.log
timeout -k 10 300 python tools/bitmap_ab.py 3 > $out/bitmap_ab.txt 2>&1 || { cat $out/bitmap_ab.txt; exit 3; }
grep -v amdgpu.ids $out/bitmap_ab.txt
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 4; }
tail -c 200 $out/bench_driver.json
