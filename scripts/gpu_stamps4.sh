set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py 4 30 1 > gpurun_out/stamps4.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 4 30 5 > gpurun_out/stamps4_b2b.log 2>&1 || exit $?
cat gpurun_out/stamps4.log gpurun_out/stamps4_b2b.log
