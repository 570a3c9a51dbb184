set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for W in 2 3; do
JSP_LIB_PATH=$PWD/tools/diag/libjsplace_pw$W.so timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/pw$W.txt 2>&1 || exit $?
echo "pipe waves $W"; grep "cfg5:\|cfg3:" gpurun_out/pw$W.txt
done
timeout -k 10 240 python3 tools/host_api_probe.py > gpurun_out/pw4.txt 2>&1 || exit $?
echo "pipe waves 4"; grep "cfg5:\|cfg3:" gpurun_out/pw4.txt
