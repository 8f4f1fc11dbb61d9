#!/bin/bash
# One GPU session on the box: parity tests, smoke, bench, rocprofv3 kernel-trace summary of the
# bench, PMC traffic passes.  Every GPU step runs under its own time limit; the session stops at
# the first step that ends abnormally (fault / abort / timeout: exit status > 1); a plain test
# failure (pytest exit 1) is recorded and the later steps still run.
#   STEPS=pytest,smoke,bench,prof,traffic  PYTEST_ARGS=...  BENCH_ARGS=...  TAG=r02
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_or_stop() {  # $1 = exit code, $2 = step name
  local rc=$1
  echo "[$2] exit $rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after abnormal exit of $2"; exit "$rc"; fi
}
STEPS=${STEPS:-pytest,smoke,bench,prof,traffic}
if [[ $STEPS == *pytest* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/${TAG}_pytest_gpu.log" 2>&1
  ok_or_stop $? pytest
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1
  ok_or_stop $? smoke
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/${TAG}_bench.log" 2>&1
  ok_or_stop $? bench
fi
if [[ $STEPS == *prof* ]]; then
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/${TAG}_bench_prof.log" 2>&1)
  ok_or_stop $? prof
fi
if [[ $STEPS == *traffic* ]]; then
  timeout -k 10 900 python tools/pmc_traffic.py "$OUT/${TAG}_traffic.json" ${BENCH_ARGS:-} > "$OUT/${TAG}_traffic.log" 2>&1
  ok_or_stop $? traffic
fi
exit 0
