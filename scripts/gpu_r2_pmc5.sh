set -u
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$R/gpurun_out/pmc5a" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 5 --steps 10 --fused 0 > "$R/gpurun_out/pmc5a.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC -d "$R/gpurun_out/pmc5b" -o run --output-format csv -- python3 "$R/tools/run_cfg.py" --cfg 5 --steps 10 --fused 0 > "$R/gpurun_out/pmc5b.log" 2>&1 || exit $?
echo done
