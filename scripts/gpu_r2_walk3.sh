set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps_walk.py 5 1 20 > gpurun_out/walkstamps5.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps_words.py 5 1 20 > gpurun_out/walkwords5.log 2>&1 || exit $?
cat gpurun_out/walkstamps5.log gpurun_out/walkwords5.log
