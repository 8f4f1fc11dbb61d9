#!/bin/bash
# One GPU session: parity tests, smoke, PMC traffic passes, bench, rocprofv3 kernel-trace
# summary.  Stops at the first step that dies abnormally (fault / abort / timeout); plain
# test failures (pytest exit 1) are recorded and the later steps still run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_or_stop() {  # $1 = exit code, $2 = step name
  local rc=$1
  echo "[$2] exit $rc" | tee -a "$OUT/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after abnormal exit of $2"; exit "$rc"; fi
}
STEPS=${STEPS:-pytest,smoke,traffic,bench,prof}
if [[ $STEPS == *pytest* ]]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  ok_or_stop $? pytest
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  ok_or_stop $? smoke
fi
if [[ $STEPS == *traffic* ]]; then
  timeout -k 10 900 python tools/pmc_traffic.py "$OUT/hbm_traffic.json" ${BENCH_ARGS:-} > "$OUT/traffic.log" 2>&1
  ok_or_stop $? traffic
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py --traffic-json "$OUT/hbm_traffic.json" ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
  ok_or_stop $? bench
fi
if [[ $STEPS == *prof* ]]; then
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --traffic-json "$OUT/hbm_traffic.json" ${BENCH_ARGS:-} > "$OUT/bench_prof.log" 2>&1)
  ok_or_stop $? prof
fi
if [[ $STEPS == *diag* ]]; then
  timeout -k 10 300 python tools/diag.py 1024 ${DIAG_VARIANT:-0} > "$OUT/diag.log" 2>&1
  ok_or_stop $? diag
fi
if [[ $STEPS == *ab* ]]; then
  timeout -k 10 300 python tools/ab.py --variants ${AB_VARIANTS:-0,2,5,6} --rounds 10 > "$OUT/ab.log" 2>&1
  ok_or_stop $? ab
fi
if [[ $STEPS == *latency* ]]; then
  timeout -k 10 300 python tools/latency_probe.py > "$OUT/latency.log" 2>&1
  ok_or_stop $? latency
fi
exit 0
