#!/bin/bash
# waker spin A/B (slept host), service tests
out=gpurun_out/r4/${1:-p20}
mkdir -p $out
timeout -k 10 120 python tools/cold_probe3.py 40 slept > $out/cold_spin20.txt 2>&1 || exit 3
JSP_WAKER_SPIN_MS=0 timeout -k 10 120 python tools/cold_probe3.py 40 slept > $out/cold_spin0.txt 2>&1 || exit 3
timeout -k 10 120 python tools/cold_probe3.py 40 slept > $out/cold_spin20b.txt 2>&1 || exit 3
JSP_WAKER_SPIN_MS=0 timeout -k 10 120 python tools/cold_probe3.py 40 slept > $out/cold_spin0b.txt 2>&1 || exit 3
timeout -k 10 300 python -u -m pytest tests/test_service_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_svc.log 2>&1 || exit 2
