# Round-2 final evidence: GPU parity (all), smoke, the bench line, its
# rocprofv3 kernel trace, PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) on configs
# 2, 4, 5, the streaming ceiling, the service phase probe and host-API probe.
# Every GPU step is time-limited; stop at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${PROF_TAG:-final}"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
echo bench-ok
timeout -k 10 120 tools/diag/stream_ceiling > "$OUT/stream_ceiling.json" 2> "$OUT/stream_ceiling.err" || exit $?
timeout -k 10 200 python3 tools/svc_probe.py 2000 > "$OUT/svc_probe.txt" 2>&1 || exit $?
timeout -k 10 240 python3 tools/host_api_probe.py > "$OUT/host_api_phases.txt" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/bench_trace" -o run --output-format csv -- python3 "$R/bench.py" --trials 100 --cpu-seconds 0 > "$OUT/bench_trace.log" 2>&1 || exit $?
echo trace-ok
for cfg in 2 4 5; do
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20 > "$OUT/pmc_fetch$cfg.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20 > "$OUT/pmc_write$cfg.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/pmc_sq$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20 > "$OUT/pmc_sq$cfg.log" 2>&1 || exit $?
done
python3 "$R/tools/summarize_prof.py" "$OUT" > "$OUT/summary.txt" 2>&1
echo all-done
