#!/bin/bash
# Round-6 GPU session 3: parity of the tree's library (one gather per pass + in-kernel replay), the
# drain-pass segments of both pass structures, and the A/B against the round-5 design.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_counters.py tests/test_gpu_fullsize.py \
  -m gpu -x -q -rf --timeout 240 --timeout-method thread > "$OUT/pytest_parity.log" 2>&1
rc=$?; echo "parity rc $rc"; tail -2 "$OUT/pytest_parity.log"; [ $rc -ne 0 ] && exit $rc
for v in seg seg0; do
  timeout -k 10 300 python -u tools/with_lib.py exp_libs/$v/libwgrt.so tools/segments.py --out "$OUT/pass_segments_$v.json" \
    > "$OUT/segments_$v.log" 2>&1
  rc=$?; echo "segments $v rc $rc"; [ $rc -ne 0 ] && exit $rc
done
for spec in C3 C3/8 C2 C4; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py base5 irep tree --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
