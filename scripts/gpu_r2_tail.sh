set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_service_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_pytest.log 2>&1 || { tail -40 gpurun_out/tail_pytest.log; exit 1; }
tail -2 gpurun_out/tail_pytest.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_placement_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_pytest2.log 2>&1 || { tail -40 gpurun_out/tail_pytest2.log; exit 1; }
tail -2 gpurun_out/tail_pytest2.log
timeout -k 10 120 python tools/stamps_walk.py 5 1 20 > gpurun_out/walkstamps5.log 2>&1 || exit $?
head -4 gpurun_out/walkstamps5.log
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/tail_hostapi.txt 2>&1 || exit $?
cat gpurun_out/tail_hostapi.txt
