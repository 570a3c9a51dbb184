#!/bin/bash
out=gpurun_out/r5/${1:-p15}
mkdir -p $out
for i in 1 2; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_$i.json 2> $out/bench_$i.err || { tail -20 $out/bench_$i.err; exit 4; }
  tail -c 150 $out/bench_driver_$i.json
done
