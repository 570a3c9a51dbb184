#!/bin/bash
# C-timed host-API loops: GPU suite, cold probe, driver bench twice
out=gpurun_out/r5/${1:-p5}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 2; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python tools/cold_probe4.py 30 > $out/cold4_product.txt 2>&1 || exit 3
grep -v amdgpu.ids $out/cold4_product.txt
for i in 1 2; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_$i.json 2> $out/bench_$i.err || { tail -20 $out/bench_$i.err; exit 4; }
  tail -c 300 $out/bench_driver_$i.json
done
