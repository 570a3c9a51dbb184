#!/bin/bash
out=gpurun_out/r4/${1:-p28}
mkdir -p $out
timeout -k 10 200 python tools/bar_ab.py 3 > $out/bar_ab.txt 2>&1 || exit 7
timeout -k 10 120 python tools/stop_probe.py > $out/stop_spin.txt 2>&1 || exit 3
JSP_SVC_STOP_SPIN=0 timeout -k 10 120 python tools/stop_probe.py > $out/stop_block.txt 2>&1 || exit 3
JSP_SVC_BAR=1 timeout -k 10 300 python -u -m pytest tests/test_service_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_svc_bar.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 2
