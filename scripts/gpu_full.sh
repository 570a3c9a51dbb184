# tests + smoke + bench + kernel trace + PMC passes (each GPU step time-limited, stop on fault)
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o run --output-format csv -- python3 "$R/bench.py" --trials 0 --cpu-seconds 0 > "$R/gpurun_out/prof_bench.log" 2>&1 || exit $?
for cfg in 2 4; do
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$R/gpurun_out/pmc_sq$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20 > "$R/gpurun_out/pmc_sq$cfg.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20 > "$R/gpurun_out/pmc_fetch$cfg.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20 > "$R/gpurun_out/pmc_write$cfg.log" 2>&1 || exit $?
done
echo all-done
