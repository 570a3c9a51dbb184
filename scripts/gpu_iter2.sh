# GPU parity tests, per-kernel breakdown of every config, tally/compaction stamps
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/breakdown.py > gpurun_out/breakdown.log 2>&1 || exit $?
cat gpurun_out/breakdown.log
timeout -k 10 120 python tools/stamps.py 4 30 5 > gpurun_out/stamps4_b2b.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 2 40 20 > gpurun_out/stamps2_b2b.log 2>&1 || exit $?
grep -v '  wg ' gpurun_out/stamps4_b2b.log gpurun_out/stamps2_b2b.log
