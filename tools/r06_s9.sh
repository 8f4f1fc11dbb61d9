#!/bin/bash
# Round-6 GPU session 9: where the launch tail's line-0 prefetch loses -- the library without it (nopf), the
# prediction alone (pfp3), plus the pass's vmcnt(0) (pfp2), plus the prefetch itself (tree).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s9
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in C3 C3/8; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py nopf pfp3 pfp2 tree --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
