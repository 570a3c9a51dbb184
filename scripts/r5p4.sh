#!/bin/bash
# SCHED_IDLE waker, dispatcher stamps, span + empty grid: GPU suite, service phase
# probe, cold probe (3 reps), driver bench
out=gpurun_out/r5/${1:-p4}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 2; }
tail -2 $out/pytest_gpu.log
timeout -k 10 200 python tools/svc_probe.py 500 > $out/svc_probe.txt 2>&1 || exit 3
grep -v amdgpu.ids $out/svc_probe.txt
for i in 1 2 3; do
  timeout -k 10 120 python tools/cold_probe4.py 30 > $out/cold4_product_$i.txt 2>&1 || exit 3
done
cat $out/cold4_*.txt | grep -v amdgpu.ids
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 4; }
tail -c 300 $out/bench_driver.json
