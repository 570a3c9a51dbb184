# Copy one GPU run's evidence from gpurun_out/TAG into profiles/ROUND/NAME
# (tracked): rocprofv3 summaries and kernel stats, PMC counter csvs renamed to
# the names bench.py looks up (pmc_{fetch,write,sq}_cfgN.csv), bench lines,
# probe outputs, test and smoke logs.
#   bash scripts/collect_profiles.sh TAG ROUND/NAME
set -eu
src="gpurun_out/$1"; dst="profiles/$2"
mkdir -p "$dst"
for f in summary.txt bench_driver.json bench.json stream_ceiling.json svc_probe.txt host_api_phases.txt \
         smoke.log gpus2.log mailbox_probe.json valu_rate.json; do
    [ -f "$src/$f" ] && cp "$src/$f" "$dst/"
done
for f in "$src"/*.txt; do [ -f "$f" ] && cp "$f" "$dst/"; done
[ -f "$src/pytest_gpu.log" ] && tail -3 "$src/pytest_gpu.log" > "$dst/pytest_gpu_tail.txt"
[ -f "$src/bench_trace/run_kernel_stats.csv" ] && cp "$src/bench_trace/run_kernel_stats.csv" "$dst/bench_kernel_stats.csv"
for kind in fetch write sq; do
    for d in "$src"/pmc_${kind}[0-9]*; do
        [ -d "$d" ] || continue
        n="${d##*pmc_${kind}}"
        [ -f "$d/run_counter_collection.csv" ] && cp "$d/run_counter_collection.csv" "$dst/pmc_${kind}_cfg${n}.csv"
    done
done
echo "$2" > profiles/LATEST
ls "$dst"
