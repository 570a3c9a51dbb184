#!/bin/bash
out=gpurun_out/r4/${1:-p25}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "level or fold or config or cfg4" > $out/pytest_level.log 2>&1 || exit 2
for i in 1 2; do
timeout -k 10 120 python tools/cfg4_step.py > $out/step_xcd_$i.txt 2>&1 || exit 3
JSP_LEVEL_XCD=0 timeout -k 10 120 python tools/cfg4_step.py > $out/step_spread_$i.txt 2>&1 || exit 3
done
timeout -k 10 120 python tools/stamps_level.py 30 > $out/stamps_level.txt 2>&1 || exit 5
