set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/g2_hostapi.txt 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 2 60 1 > gpurun_out/g2_stamps2_idle.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py 2 60 20 > gpurun_out/g2_stamps2_b2b.log 2>&1 || exit $?
echo done
