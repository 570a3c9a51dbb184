#!/bin/bash
out=gpurun_out/r5/${1:-p13}
mkdir -p $out
timeout -k 10 300 python tools/gap_probe.py > $out/gap.txt 2>&1 || { cat $out/gap.txt; exit 3; }
timeout -k 10 300 python tools/gap_probe.py svc_entries=1 >> $out/gap.txt 2>&1 || { cat $out/gap.txt; exit 3; }
grep -v amdgpu.ids $out/gap.txt
