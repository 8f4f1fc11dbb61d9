#!/bin/bash
# Round-6 GPU session 18: the single-trace grid rule K (workgroups = ceil(K sqrt(work items))) re-measured on
# the final library: K = 5.5 / 6.5 (the product) / 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s18
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in C3 C3/8 C2 C4; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py tree+grid_sqrt_k=5.5 tree tree+grid_sqrt_k=8 --rounds 4 --config $c --shard $sh \
    > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
