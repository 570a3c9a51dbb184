#!/bin/bash
out=gpurun_out/r5/${1:-p14}
mkdir -p $out
lscpu > $out/lscpu.txt 2>&1 || true
timeout -k 10 300 python tools/numa_probe.py > $out/numa.txt 2>&1 || { cat $out/numa.txt; exit 3; }
grep -v amdgpu.ids $out/numa.txt
grep -E "NUMA|Socket|Model name" $out/lscpu.txt
