#!/bin/bash
# Round-4 small-batch A/B: GPU parity of the tree's library (TESTS), then tools/ab.py over the small-batch
# selection (never / auto / always) on C2, the C3 shards of 8, 4 and 2 ranks, and C3.  Each step under its
# own time limit; stops at the first failure.
# (Ran on a build that added trace_jones_small_kernel and wgrt_debug_opts.small_batch; both were removed
# after this A/B without being committed, so the script no longer runs as is.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
TAG=${TAG:-r04sb}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 240 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; echo "pytest rc $rc"; tail -3 "$OUT/${TAG}_pytest.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
NAMES=${NAMES:-"tree+dbg_small_batch=-1 tree tree+dbg_small_batch=1"}
for spec in ${CASES:-C2:1 C3:8 C3:4 C3:2 C3:1}; do
  c=${spec%%:*}; n=${spec##*:}
  timeout -k 10 600 python tools/ab.py $NAMES --rounds ${ROUNDS:-4} --config $c --shard $n --fused 2 > "$OUT/${TAG}_ab_${c}_s$n.log" 2>&1
  rc=$?; echo "ab $c shard $n rc $rc"; grep SUMMARY "$OUT/${TAG}_ab_${c}_s$n.log"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/${TAG}_ab_${c}_s$n.log"; exit $rc; fi
done
exit 0
