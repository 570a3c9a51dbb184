#!/bin/bash
# device-path shapes; waker CPU exclusion A/B at 100 trials
out=gpurun_out/r5/${1:-p7}
mkdir -p $out
timeout -k 10 200 python tools/devpath_probe.py > $out/devpath.txt 2>&1 || { cat $out/devpath.txt; exit 3; }
grep -v amdgpu.ids $out/devpath.txt
for i in 1 2; do
  timeout -k 10 200 python tools/cold_probe4.py 100 > $out/cold4_product_$i.txt 2>&1 || exit 3
  JSP_LIB_PATH=tools/bin/ab_waker_anycpu/libjsplace.so timeout -k 10 200 python tools/cold_probe4.py 100 > $out/cold4_anycpu_$i.txt 2>&1 || exit 3
done
cat $out/cold4_*.txt | grep -v amdgpu.ids
