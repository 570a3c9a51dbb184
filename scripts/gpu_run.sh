# One parameterised GPU run (replaces the round-1/2 one-off scripts).
#   bash scripts/gpu_run.sh TAG STEP [STEP ...]
# Output goes to gpurun_out/TAG/. Steps, in the order given:
#   tests     pytest -m gpu (one process, per-test timeout)
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py (default flags) -> bench.json
#   driver    python bench.py --gpus 1 --steps 20 --warmup 5 (the driver's flags) -> bench_driver.json
#   gpus2     python bench.py --gpus 2 on this 1-GPU box must exit non-zero (no silent 1-GPU line)
#   ceiling   tools/bin/stream_ceiling (read / copy ceilings at the kernels' byte counts)
#   bin:NAME  tools/bin/NAME (a compiled probe) -> NAME.json
#   probes    tools/svc_probe.py + tools/host_api_probe.py
#   devloop   tools/devpath_loop.py (device paths and host API of cfg5, cfg3)
#   trace     rocprofv3 --kernel-trace --stats of the bench (no CPU legs)
#   pmc       separate rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / SQ) on configs 2, 4, 5
#   py:FILE[:ARG]  python FILE ARG (a probe under tools/) -> FILE_ARG.txt
#   pytest:SEL     pytest SEL -m gpu (one file or node id)
#   tracepy:NAME:FILE[:ARG]  rocprofv3 --kernel-trace --stats of python FILE ARG -> NAME/ (+ NAME_summary.txt)
# Every GPU step runs under its own time limit; the script stops at the first
# failure, time-out or crash (nothing further touches the GPU).
set -u
TAG="$1"; shift
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
run() {  # run SECONDS LOG CMD...
    local t="$1" log="$2"; shift 2
    timeout -k 10 "$t" "$@" > "$log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "FAILED ($rc): $*"; tail -40 "$log"; exit $rc; fi
}
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    tests)   run 900 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
             tail -2 "$OUT/pytest_gpu.log" ;;
    smoke)   run 300 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"; cat "$OUT/smoke.log" ;;
    bench)   run 500 "$OUT/bench.json" python bench.py; tail -c 600 "$OUT/bench.json" ;;
    driver)  run 500 "$OUT/bench_driver.json" python bench.py --gpus 1 --steps 20 --warmup 5; tail -c 400 "$OUT/bench_driver.json" ;;
    gpus2)   timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > "$OUT/gpus2.log" 2>&1
             rc=$?; echo "bench.py --gpus 2 exit code $rc" >> "$OUT/gpus2.log"; tail -2 "$OUT/gpus2.log"
             if [ $rc -eq 0 ] || [ $rc -ge 124 ]; then echo "FAILED: --gpus 2 should fail loudly"; exit 1; fi ;;
    ceiling) run 120 "$OUT/stream_ceiling.json" tools/bin/stream_ceiling; cat "$OUT/stream_ceiling.json" ;;
    bin:*)   b="${step#bin:}"; run 120 "$OUT/$b.json" "tools/bin/$b"; cat "$OUT/$b.json" ;;
    probes)  run 200 "$OUT/svc_probe.txt" python3 tools/svc_probe.py 2000
             run 240 "$OUT/host_api_phases.txt" python3 tools/host_api_probe.py ;;
    devloop) run 300 "$OUT/devpath_loop.txt" python3 tools/devpath_loop.py 5,3 3; cat "$OUT/devpath_loop.txt" ;;
    trace)   ( cd /tmp && export TMPDIR=/tmp && run 500 "$OUT/bench_trace.log" rocprofv3 --kernel-trace --stats -d "$OUT/bench_trace" -o run --output-format csv -- python3 "$R/bench.py" --trials 100 --cold-trials 0 --cpu-seconds 0 ) || exit $?
             python3 tools/summarize_prof.py "$OUT" > "$OUT/summary.txt" 2>&1 ;;
    pmc)     ( cd /tmp && export TMPDIR=/tmp
               for cfg in 2 4 5; do
                 run 120 "$OUT/pmc_fetch$cfg.log" rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20
                 run 120 "$OUT/pmc_write$cfg.log" rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20
                 run 120 "$OUT/pmc_sq$cfg.log" rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/pmc_sq$cfg" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg $cfg --steps 20
               done ) || exit $?
             python3 tools/summarize_prof.py "$OUT" > "$OUT/summary.txt" 2>&1 ;;
    py:*)    spec="${step#py:}"; f="${spec%%:*}"; arg=""; [ "$spec" != "$f" ] && arg="${spec#*:}"; arg="${arg//:/ }"
             log="$OUT/$(basename "$f" .py)${arg:+_${arg// /_}}.txt"
             run 600 "$log" python3 -u "$f" $arg; tail -30 "$log" ;;
    tracepy:*) spec="${step#tracepy:}"; name="${spec%%:*}"; rest="${spec#*:}"; f="${rest%%:*}"; arg=""
             [ "$rest" != "$f" ] && arg="${rest#*:}"; arg="${arg//:/ }"
             ( cd /tmp && export TMPDIR=/tmp && run 300 "$OUT/$name.log" rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- python3 "$R/$f" $arg ) || exit $?
             python3 tools/summarize_prof.py "$OUT/$name" > "$OUT/${name}_summary.txt" 2>&1; tail -25 "$OUT/${name}_summary.txt" ;;
    pytest:*) sel="${step#pytest:}"; run 900 "$OUT/pytest_$(echo "$sel" | tr '/:' '__').log" python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread
             tail -3 "$OUT/pytest_$(echo "$sel" | tr '/:' '__').log" ;;
    *)       echo "unknown step $step"; exit 2 ;;
  esac
done
echo all-done
