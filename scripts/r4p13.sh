#!/bin/bash
# one-launch level walk: A/B step times, engine GPU tests, kernel trace of the steps
out=gpurun_out/r4/${1:-p19}
mkdir -p $out
timeout -k 10 120 python tools/cfg4_step.py > $out/cfg4_step_one.txt 2>&1 || exit 3
JSP_LEVEL_ONE_LAUNCH=0 timeout -k 10 120 python tools/cfg4_step.py > $out/cfg4_step_two.txt 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_multi_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_engine.log 2>&1 || exit 2
