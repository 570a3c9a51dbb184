# PMC + kernel-trace passes of the tally / fused kernels (separate --pmc passes, no trace domains mixed in)
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pmc_trace4" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 4 --steps 20 > "$R/gpurun_out/pmc_trace4.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$R/gpurun_out/pmc_sq4" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 4 --steps 20 > "$R/gpurun_out/pmc_sq4.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch4" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 4 --steps 20 > "$R/gpurun_out/pmc_fetch4.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write4" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 4 --steps 20 > "$R/gpurun_out/pmc_write4.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$R/gpurun_out/pmc_sq2" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 2 --steps 20 > "$R/gpurun_out/pmc_sq2.log" 2>&1 || exit $?
echo pmc-done
