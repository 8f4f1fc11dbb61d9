#!/bin/bash
# Round-4 A/B session: GPU parity of the tree's library (TESTS), then tools/ab.py over NAMES on each of
# CONFIGS (C5 with 2 launches / 2 fused).  Every step under its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
TAG=${TAG:-r04ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 240 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; echo "pytest rc $rc"; tail -3 "$OUT/${TAG}_pytest.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for c in ${CONFIGS:-C3}; do
  extra=""
  if [ "$c" = "C5" ]; then extra="--launches 2 --fused 2"; fi
  timeout -k 10 600 python tools/ab.py $NAMES --rounds ${ROUNDS:-4} --config $c $extra > "$OUT/${TAG}_ab_$c.log" 2>&1
  rc=$?; echo "ab $c rc $rc"; grep SUMMARY "$OUT/${TAG}_ab_$c.log"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/${TAG}_ab_$c.log"; exit $rc; fi
done
exit 0
