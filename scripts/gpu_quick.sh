# GPU tests + bench + stamps timeline (no PMC)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --trials 300 --cpu-seconds 3 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 2 60 > gpurun_out/stamps2.log 2>&1 || exit $?
echo quick-done
