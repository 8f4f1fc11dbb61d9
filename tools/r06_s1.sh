#!/bin/bash
# Round-6 GPU session 1: the new gather test, parity of the in-kernel-replay build, the drain-pass
# segment stamps (tools/segments.py on exp_libs/seg), and the A/B of the in-kernel replay.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q -rf --timeout 120 --timeout-method thread \
  > "$OUT/pytest_dist.log" 2>&1
rc=$?; echo "pytest dist rc $rc"; tail -2 "$OUT/pytest_dist.log"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u tools/with_lib.py exp_libs/irep/libwgrt.so -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_counters.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/parity_irep.log" 2>&1
rc=$?; echo "parity irep rc $rc"; tail -2 "$OUT/parity_irep.log"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/with_lib.py exp_libs/seg/libwgrt.so tools/segments.py --out "$OUT/pass_segments.json" \
  > "$OUT/segments.log" 2>&1
rc=$?; echo "segments rc $rc"; tail -4 "$OUT/segments.log"; [ $rc -ne 0 ] && exit $rc
for spec in C3 C3/8 C2 C4; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 400 python tools/ab.py tree irep --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
