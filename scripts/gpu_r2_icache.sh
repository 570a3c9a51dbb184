# instruction-cache counters of the cfg5 fused kernel (one PMC pass per group)
set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/icache
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/icache/avail.txt" 2>&1
grep -io "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*\|SQ_WAIT_INST[A-Z_]*" "$R/gpurun_out/icache/avail.txt" | sort -u > "$R/gpurun_out/icache/names.txt"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES -d "$R/gpurun_out/icache/p1" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 5 --steps 20 > "$R/gpurun_out/icache/p1.log" 2>&1
echo rc=$?
