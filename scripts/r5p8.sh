#!/bin/bash
# parked service: GPU service tests, cold probe default vs parked, driver bench
out=gpurun_out/r5/${1:-p8}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_svc.log 2>&1 || { tail -60 $out/pytest_svc.log; exit 2; }
tail -2 $out/pytest_svc.log
for m in x parked; do
  timeout -k 10 200 python tools/cold_probe4.py 100 2 $m > $out/cold4_$m.txt 2>&1 || exit 3
done
cat $out/cold4_*.txt | grep -v amdgpu.ids
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 4; }
tail -c 300 $out/bench_driver.json
