mkdir -p gpurun_out/r4/p1
timeout -k 10 120 ./tools/bin/block_probe 15 > gpurun_out/r4/p1/block_probe.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/p1/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/p1/bench.json 2> gpurun_out/r4/p1/bench.err || exit 3
