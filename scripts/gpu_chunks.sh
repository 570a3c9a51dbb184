# Parity tests, bench, and a per-kernel breakdown of cfg4 across tally chunks-per-workgroup
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in 1 2 3 4 8; do
  echo "chunks=$c" >> gpurun_out/chunks.log
  JSP_BLOCK_CHUNKS=$c timeout -k 10 120 python tools/breakdown.py 4 >> gpurun_out/chunks.log 2>&1 || exit $?
done
cat gpurun_out/chunks.log
timeout -k 10 300 python bench.py --trials 300 --cpu-seconds 2 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
