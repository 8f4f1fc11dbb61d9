#!/bin/bash
# Round-6 GPU session 11: issue priority for the launch tail's waves (s_setprio 1 / 3 at the tail loop's entry).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s11
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in C3 C3/8 C2 C4; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py tree prio1 prio3 --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
