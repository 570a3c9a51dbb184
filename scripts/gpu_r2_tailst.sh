set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps_walk.py 5 1 20 > gpurun_out/tailst5.log 2>&1 || exit $?
grep "row 400" gpurun_out/tailst5.log
