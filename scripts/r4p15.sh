#!/bin/bash
out=gpurun_out/r4/${1:-p21}
mkdir -p $out
for i in 1 2; do
timeout -k 10 120 python tools/cfg4_step.py > $out/step_late_$i.txt 2>&1 || exit 3
JSP_LEVEL_EARLY=1 timeout -k 10 120 python tools/cfg4_step.py > $out/step_early_$i.txt 2>&1 || exit 3
done
JSP_LEVEL_EARLY=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "cfg4 or level or fold or config" > $out/pytest_early.log 2>&1 || exit 2
