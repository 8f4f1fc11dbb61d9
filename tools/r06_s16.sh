#!/bin/bash
# Round-6 GPU session 16: the launch tail retires finished traces at the end of the pass (their stores behind the pass's loads) against the library without it; parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s16
mkdir -p "$OUT"
export TMPDIR=/tmp WGRT_RESULTS_DIR=$OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_counters.py tests/test_gpu_fullsize.py -m gpu -x -q -rf \
  --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for spec in C3 C3/8 C2 C4 C3/4; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py nolr tree --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
