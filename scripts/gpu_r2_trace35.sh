# kernel traces of configs 3 and 5 in both launch shapes
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/t35
cd /tmp && export TMPDIR=/tmp
for cfg in 3 5; do for fu in 1 0; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/t35/c${cfg}f${fu}" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 50 --fused $fu > "$R/gpurun_out/t35/c${cfg}f${fu}.log" 2>&1 || exit $?
done; done
python3 "$R/tools/summarize_prof.py" "$R/gpurun_out/t35" > "$R/gpurun_out/t35/summary.txt"
echo done
