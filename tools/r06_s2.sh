#!/bin/bash
# Round-6 GPU session 2: drain-pass segment stamps (fixed attribution), then the full GPU suite on the
# tree's library (in-kernel replay on by default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/with_lib.py exp_libs/seg/libwgrt.so tools/segments.py --out "$OUT/pass_segments.json" \
  > "$OUT/segments.log" 2>&1
rc=$?; echo "segments rc $rc"; tail -3 "$OUT/segments.log" | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 "$OUT/pytest_gpu.log"
exit $rc
