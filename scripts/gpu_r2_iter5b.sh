# GPU parity suite, cfg5 stamps, and the streaming-ceiling probe
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/stamps_walk.py 5 1 20 > gpurun_out/walkstamps5.log 2>&1 || exit $?
cat gpurun_out/walkstamps5.log
timeout -k 10 120 tools/diag/stream_ceiling > gpurun_out/stream_ceiling.json 2> gpurun_out/stream_ceiling.err || exit $?
cat gpurun_out/stream_ceiling.json
echo all-done
