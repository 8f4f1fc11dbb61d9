#!/bin/bash
# A/B of single-trace grid rules (exp_libs builds, tools/ab_build.py): tools/ab.py on C3 and C2,
# then every build's emulated strong-scaling shards of C3 (bench.py --emulate-ranks 2 / 4 / 8).
#   NAMES="base k55 k65"  TAG=r03gk  bash tools/grid_session.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
TAG=${TAG:-gk}
NAMES=${NAMES:-base}
mkdir -p $O
timeout -k 10 400 python tools/ab.py $NAMES --rounds 3 --config C3 --fused 4 > $O/${TAG}_ab_C3.log 2>&1 || exit $?
grep SUMMARY $O/${TAG}_ab_C3.log
timeout -k 10 300 python tools/ab.py $NAMES --rounds 3 --config C2 --fused 4 > $O/${TAG}_ab_C2.log 2>&1 || exit $?
grep SUMMARY $O/${TAG}_ab_C2.log
for v in $NAMES; do
  for n in 2 4 8; do
    timeout -k 10 200 python tools/with_lib.py $(pwd)/exp_libs/$v/libwgrt.so bench.py --emulate-ranks $n --steps 10 --warmup 2 \
      > $O/${TAG}_em_${v}_$n.log 2>&1 || exit $?
    echo "$v N=$n $(grep -o '"predicted_ms_per_step": [0-9.]*' $O/${TAG}_em_${v}_$n.log)"
  done
done
