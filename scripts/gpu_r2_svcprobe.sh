set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python3 tools/svc_probe.py 2000 > gpurun_out/svc_probe.txt 2>&1 || { cat gpurun_out/svc_probe.txt; exit 1; }
cat gpurun_out/svc_probe.txt
