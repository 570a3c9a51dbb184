#!/bin/bash
# deferred waker notify + CPU exclusion A/B, bracket probe
out=gpurun_out/r5/${1:-p6}
mkdir -p $out
timeout -k 10 120 python tools/bracket_probe.py 40 > $out/bracket.txt 2>&1 || exit 3
grep -v amdgpu.ids $out/bracket.txt
for i in 1 2; do
  timeout -k 10 120 python tools/cold_probe4.py 40 > $out/cold4_product_$i.txt 2>&1 || exit 3
  JSP_LIB_PATH=tools/bin/ab_waker_anycpu/libjsplace.so timeout -k 10 120 python tools/cold_probe4.py 40 > $out/cold4_anycpu_$i.txt 2>&1 || exit 3
done
cat $out/cold4_*.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "service or patch or wake" > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 2; }
tail -2 $out/pytest_gpu.log
