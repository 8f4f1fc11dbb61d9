cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 400 python tools/ab.py base k45 k55 k65 --rounds 3 --config C3 --fused 4 > $O/r03gk_ab_C3.log 2>&1 || exit $?
grep SUMMARY $O/r03gk_ab_C3.log
timeout -k 10 300 python tools/ab.py base k45 k55 k65 --rounds 3 --config C2 --fused 4 > $O/r03gk_ab_C2.log 2>&1 || exit $?
grep SUMMARY $O/r03gk_ab_C2.log
for v in base k45 k55 k65; do
  for n in 2 4 8; do
    WGRT_LIB=$GRAFT_REPO_ROOT/exp_libs/$v/libwgrt.so timeout -k 10 200 python bench.py --emulate-ranks $n --steps 10 --warmup 2 > $O/r03gk_em_${v}_$n.log 2>&1 || exit $?
    echo "$v N=$n $(grep -o '"predicted_ms_per_step": [0-9.]*' $O/r03gk_em_${v}_$n.log)"
  done
done
