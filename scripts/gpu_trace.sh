# Kernel traces of cfg4 / cfg2 (product build) + HBM PMC passes of cfg2's compaction kernel and cfg4's tally
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in 4 2; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace$c" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $c --steps 50 > "$R/gpurun_out/trace$c.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch$c" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $c --steps 20 > "$R/gpurun_out/pmc_fetch$c.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write$c" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $c --steps 20 > "$R/gpurun_out/pmc_write$c.log" 2>&1 || exit $?
done
cd "$R"; python tools/summarize_prof.py gpurun_out > gpurun_out/trace_summary.txt; cat gpurun_out/trace_summary.txt
