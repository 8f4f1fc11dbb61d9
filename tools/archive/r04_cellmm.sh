cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for c in C3 C4 C2; do
  extra=""
  timeout -k 10 500 python tools/ab.py tree tree@cell_mm=0.015625 tree@cell_mm=0.03125 tree@cell_mm=0.0625 --rounds 3 --config $c --fused 10 > gpurun_out/r04_ab_cellmm_$c.log 2>&1
  rc=$?; echo "ab $c rc $rc"; grep SUMMARY gpurun_out/r04_ab_cellmm_$c.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/r04_ab_cellmm_$c.log; exit $rc; fi
done
