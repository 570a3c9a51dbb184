#!/bin/bash
# micro-patches in the request line + paced stream queries: service and engine
# GPU tests, patched-step probe, cold probe A/B (waker vs inline), link floor, driver bench
out=gpurun_out/r5/${1:-p2}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_svc_engine.log 2>&1 || { tail -40 $out/pytest_svc_engine.log; exit 2; }
tail -2 $out/pytest_svc_engine.log
timeout -k 10 120 python tools/patched_probe.py 400 > $out/patched_probe.txt 2>&1 || exit 3
cat $out/patched_probe.txt | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 120 python tools/cold_probe4.py 30 > $out/cold4_product_$i.txt 2>&1 || exit 3
  JSP_LIB_PATH=$PWD/tools/bin/ab_inlinewake/libjsplace.so timeout -k 10 120 python tools/cold_probe4.py 30 > $out/cold4_inline_$i.txt 2>&1 || exit 3
done
cat $out/cold4_*.txt | grep -v amdgpu.ids
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 4; }
tail -c 300 $out/bench_driver.json
