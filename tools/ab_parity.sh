#!/bin/bash
# A/B session: GPU tests of the tree's library (TESTS, optional), GPU parity of each
# exp_libs build in PARITY (tests/test_gpu_parity.py + test_gpu_counters.py), then tools/ab.py over
# NAMES on each SPEC of SPECS ("C3", "C3/8" = rank 0's interleaved shard of 8, "C5" short).  Every step
# under its own time limit; stops at the first abnormal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_tree.log" 2>&1
  rc=$?; echo "pytest tree rc $rc"; tail -3 "$OUT/pytest_tree.log"
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
for v in $PARITY; do
  timeout -k 10 400 python -u tools/with_lib.py exp_libs/$v/libwgrt.so -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_counters.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/parity_$v.log" 2>&1
  rc=$?; echo "parity $v rc $rc"; tail -2 "$OUT/parity_$v.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for spec in ${SPECS:-C3}; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  extra=""
  if [ "$c" = "C5" ] || [ "$c" = "C5d" ]; then extra="--launches 2 --fused 2"; fi
  tag=${c}_s$sh
  timeout -k 10 600 python tools/ab.py $NAMES --rounds ${ROUNDS:-4} --config $c --shard $sh $extra > "$OUT/ab_$tag.log" 2>&1
  rc=$?; echo "ab $tag rc $rc"; grep SUMMARY "$OUT/ab_$tag.log"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/ab_$tag.log"; exit $rc; fi
done
exit 0
