#!/bin/bash
# Round-6 GPU session 6: full GPU suite (AMP instantiations, scene info ABI 7), the A/B against the round-5
# design, the driver's bench command, and a rocprofv3 kernel-trace summary of it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s6
mkdir -p "$OUT"
export TMPDIR=/tmp WGRT_RESULTS_DIR=$OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for spec in C3 C3/8 C2 C4; do
  c=${spec%/*}; sh=1; [ "$spec" != "$c" ] && sh=${spec#*/}
  timeout -k 10 500 python tools/ab.py base5 tree --rounds 4 --config $c --shard $sh > "$OUT/ab_${c}_s$sh.log" 2>&1
  rc=$?; echo "ab $spec rc $rc"; grep SUMMARY "$OUT/ab_${c}_s$sh.log"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.jsonl" 2> "$OUT/bench_driver.err"
rc=$?; echo "bench rc $rc"; [ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
   python3 "$OLDPWD/bench.py" --no-cpu-baseline --no-extras --steps 200 --warmup 5 > "$OUT/bench_prof.jsonl" 2>&1)
echo "prof rc $?"
exit 0
