#!/bin/bash
# bitmap answer: service + engine GPU tests, A/B, hop split probe
out=gpurun_out/r5/${1:-p11}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_service_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -60 $out/pytest.log; exit 2; }
tail -2 $out/pytest.log
timeout -k 10 300 python tools/bitmap_ab.py 3 > $out/bitmap_ab.txt 2>&1 || { cat $out/bitmap_ab.txt; exit 3; }
grep -v amdgpu.ids $out/bitmap_ab.txt
timeout -k 10 300 python tools/svc_probe.py 1000 > $out/svc_probe.txt 2>&1 || { cat $out/svc_probe.txt; exit 3; }
grep -v amdgpu.ids $out/svc_probe.txt
