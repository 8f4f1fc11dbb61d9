#!/bin/bash
# Round-6 GPU session 17: wave timelines on the final library (C3, rank 0 of 4 and of 8, C2), the drain
# evidence of DESIGN.md §5.2 refreshed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s17
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in C3 C3/4 C3/8 C2; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 300 python tools/timeline.py --config $c --shard $sh --out "$OUT/timeline_${c}_s$sh.json" > "$OUT/timeline_${c}_s$sh.log" 2>&1
  rc=$?; echo "timeline $spec rc $rc"; tail -3 "$OUT/timeline_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
