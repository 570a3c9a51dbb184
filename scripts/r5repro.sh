#!/bin/bash
# Round-4 red run p2/p3 reproduced on its own commit (8b50930, worktree under
# tools/repro_8b50930): the two slowest cases, default and with each path
# switch of that tree off
out=$GRAFT_REPO_ROOT/gpurun_out/r5/${1:-repro}
mkdir -p $out
cd tools/repro_8b50930
T="tests/test_engine_gpu.py::test_folded_feasibility_and_level_walk[16] tests/test_engine_gpu.py::test_folded_feasibility_and_level_walk[2]"
for sw in default JSP_NO_PIPE=1 JSP_ASSIGN_LEVEL=0 JSP_FEAS_FOLD=0; do
  if [ $sw = default ]; then e=""; else e="$sw"; fi
  echo "== $sw" >> $out/repro.txt
  env $e timeout -k 10 400 python -u -m pytest $T -m gpu -q --durations=5 --timeout 300 --timeout-method thread >> $out/repro.txt 2>&1 || { echo "rc=$? ($sw)" >> $out/repro.txt; tail -30 $out/repro.txt; exit 3; }
  grep -E "s call|passed|failed" $out/repro.txt | tail -4
done
