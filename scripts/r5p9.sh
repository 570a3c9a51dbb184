#!/bin/bash
# C-timed recovery loops: service GPU tests, driver bench x2
out=gpurun_out/r5/${1:-p9}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_svc.log 2>&1 || { tail -60 $out/pytest_svc.log; exit 2; }
tail -2 $out/pytest_svc.log
for i in 1 2; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_$i.json 2> $out/bench_$i.err || { tail -20 $out/bench_$i.err; exit 4; }
  tail -c 200 $out/bench_driver_$i.json
done
