# Same-box A/B: the product library against tools/bin/ab_prev/libjsplace.so (a build of the previous kernels),
# alternating, on configs $CFGS (default 5,3): tools/devpath_loop.py twice each, then tools/svc_probe.py.
#   TAG=name CFGS=5,3 bash scripts/ab_same_box.sh
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r6/${TAG:-ab}; mkdir -p $OUT
for v in new prev new2 prev2; do
  lib=""; case $v in prev*) lib=tools/bin/ab_prev/libjsplace.so;; esac
  JSP_LIB_PATH=$lib timeout -k 10 200 python -u tools/devpath_loop.py ${CFGS:-5,3} 2 > $OUT/devpath_$v.txt 2>&1 || { cat $OUT/devpath_$v.txt; exit 1; }
done
for v in new prev; do
  lib=""; case $v in prev*) lib=tools/bin/ab_prev/libjsplace.so;; esac
  JSP_LIB_PATH=$lib timeout -k 10 200 python -u tools/svc_probe.py 1000 ${CFGS:-5,3} > $OUT/svc_$v.txt 2>&1 || { cat $OUT/svc_$v.txt; exit 1; }
done
grep -H "cfg" $OUT/devpath_*.txt; grep -H "timing=" $OUT/svc_*.txt
