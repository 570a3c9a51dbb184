set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_service_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tail2_pytest.log 2>&1 || { tail -40 gpurun_out/tail2_pytest.log; exit 1; }
tail -2 gpurun_out/tail2_pytest.log
timeout -k 10 120 python tools/stamps_walk.py 5 1 20 > gpurun_out/walkstamps5.log 2>&1 || exit $?
head -4 gpurun_out/walkstamps5.log
timeout -k 10 200 python3 tools/tally_probe.py > gpurun_out/tally_probe.txt 2>&1 || { cat gpurun_out/tally_probe.txt; exit 1; }
cat gpurun_out/tally_probe.txt
