#!/bin/bash
# round-4: cfg4 step kernel trace, level walker A/B
out=gpurun_out/r4/${1:-p5}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 python tools/cfg4_step.py > $out/cfg4_step.txt 2>&1 || exit 1
JSP_ASSIGN_LEVEL=0 timeout -k 10 200 python tools/cfg4_step.py >> $out/cfg4_step.txt 2>&1 || exit 1
JSP_ASSIGN_LEVEL=0 JSP_FEAS_FOLD=0 timeout -k 10 200 python tools/cfg4_step.py >> $out/cfg4_step.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o cfg4 -- python tools/cfg4_step.py > $out/prof.log 2>&1 || exit 2
