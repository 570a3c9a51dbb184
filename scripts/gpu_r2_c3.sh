set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps_walk.py 3 1 20 > gpurun_out/walkstamps3.log 2>&1 || exit $?
cat gpurun_out/walkstamps3.log | head -60
