#!/bin/bash
# Round-5 GPU session 1: the round's robustness changes on the box (KArgs kernarg handle, device
# scopes, interaction counting, hand-off CAS), the out-of-line EDGE-resolution build's parity (the
# build that faulted in round 4), the bench, and the drain timelines of C3, C2 and C3's N = 4 / 8
# shards on this library.  Each GPU step under its own limit; stop at the first abnormal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05s1
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step parity_edge_noinline 400 python -u tools/with_lib.py exp_libs/edge_noinline/libwgrt.so -m pytest \
  tests/test_gpu_parity.py tests/test_gpu_counters.py -m gpu -x -q -rf --timeout 120 --timeout-method thread
step bench 400 python bench.py
for s in 1 4 8; do
  step timeline_C3_s$s 200 python tools/timeline.py --config C3 --shard $s --reps 3 --out $OUT/timeline_C3_s$s.json
done
step timeline_C2 200 python tools/timeline.py --config C2 --reps 3 --out $OUT/timeline_C2.json
exit 0
