#!/bin/bash
# Round-6 GPU session 5: the full GPU suite on the tree's library (in-kernel replay, ABI 7 libm_rays,
# amplification-tracked certification), then the A/B against the round-5 design and the tree without
# the amplification step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s5
mkdir -p "$OUT"
export TMPDIR=/tmp WGRT_RESULTS_DIR=$OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -gt 1 ] && exit $rc
for spec in C3 C3/8 C2 C4; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py base5 noamp tree --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
