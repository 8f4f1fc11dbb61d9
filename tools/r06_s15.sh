#!/bin/bash
# Round-6 GPU session 15: drain-pass segments on the final library (compiler-visible waits).
# (forced waits, LDS-accumulated sums) and the wave-uniform ones.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s15
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in seg1 seg2; do
  timeout -k 10 300 python -u tools/with_lib.py exp_libs/$v/libwgrt.so tools/segments.py --out "$OUT/pass_segments_$v.json" \
    > "$OUT/segments_$v.log" 2>&1
  rc=$?; echo "segments $v rc $rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
