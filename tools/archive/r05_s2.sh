#!/bin/bash
# Round-5 GPU session 2: all GPU tests (adversarial certification + parity, counters with forced
# replays, device scopes), then the default bench line (emulated_strong with C5d / C5 and the
# gather's cost, roofline.binding).  Each GPU step under its own limit; stop at the first abnormal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05s2}
mkdir -p $OUT
export TMPDIR=/tmp WGRT_RESULTS_DIR=$OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name"; exit $rc; fi
}
[[ ${STEPS:-pytest,bench} == *pytest* ]] && step pytest_gpu 700 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
[[ ${STEPS:-pytest,bench} == *bench* ]] && step bench 500 python bench.py ${BENCH_ARGS:-}
exit 0
