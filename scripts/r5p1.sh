#!/bin/bash
# round 5, first box: GPU suite on the switch-free library, cold-recovery phase
# probe (product waker vs inline wake, interleaved), driver-flag bench
out=gpurun_out/r5/${1:-p1}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=15 > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 2; }
tail -3 $out/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 120 python tools/cold_probe4.py 30 > $out/cold4_product_$i.txt 2>&1 || exit 3
  JSP_LIB_PATH=$PWD/tools/bin/ab_inlinewake/libjsplace.so timeout -k 10 120 python tools/cold_probe4.py 30 > $out/cold4_inline_$i.txt 2>&1 || exit 3
done
cat $out/cold4_*.txt | grep -v amdgpu.ids
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench.err || exit 4
tail -c 300 $out/bench_driver.json
