#!/bin/bash
# Round-6 GPU session 4: wave-uniform drain-pass segments of both pass structures, and the A/B of the
# structure pieces (one gather per pass, late retire) and of the amplification-tracked bound.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s4
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in seg2 seg20; do
  timeout -k 10 300 python -u tools/with_lib.py exp_libs/$v/libwgrt.so tools/segments.py --out "$OUT/pass_segments_$v.json" \
    > "$OUT/segments_$v.log" 2>&1
  rc=$?; echo "segments $v rc $rc"; [ $rc -ne 0 ] && exit $rc
done
for spec in C3 C3/8 C2; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py irep uni unil tree --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
