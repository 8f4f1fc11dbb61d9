#!/bin/bash
# One GPU session on the box: parity tests, smoke, bench, rocprofv3 kernel-trace summary of the
# bench, PMC traffic passes.  Every GPU step runs under its own time limit; the session stops at
# the first step that ends abnormally (fault / abort / timeout: exit status > 1); a plain test
# failure (pytest exit 1) is recorded and the later steps still run.
#   STEPS=pytest,smoke,bench,prof,traffic,pmc,configs,emulate,rehearsal  PYTEST_ARGS=...  BENCH_ARGS=...  TAG=r03
#   configs: bench lines of C2 / C4 / C5 / C5d; emulate: --emulate-ranks 2/4/8 (C3) and 8 (C4); rehearsal:
#   torchrun 2 ranks on the one GPU over gloo (the N > 1 code path: interleaved shards + gather)
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
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > "$OUT/${TAG}_bench_prof.log" 2>&1)
  ok_or_stop $? prof
fi
if [[ $STEPS == *traffic* ]]; then
  timeout -k 10 900 python tools/pmc_traffic.py "$OUT/${TAG}_traffic.json" ${BENCH_ARGS:-} > "$OUT/${TAG}_traffic.log" 2>&1
  ok_or_stop $? traffic
fi
if [[ $STEPS == *pmc* ]]; then
  TAG=$TAG timeout -k 10 900 bash tools/pmc_passes.sh > "$OUT/${TAG}_pmc.log" 2>&1
  ok_or_stop $? pmc
  python tools/pmc_summary.py "$OUT/${TAG}_pmc" "$OUT/${TAG}_pmc_summary.json" --merge "$OUT/${TAG}_pmc.json" \
    >> "$OUT/${TAG}_pmc.log" 2>&1
fi
if [[ $STEPS == *configs* ]]; then
  for c in C2 C4 C5 C5d; do
    timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 > "$OUT/${TAG}_bench_$c.log" 2>&1
    ok_or_stop $? bench_$c
  done
fi
if [[ $STEPS == *emulate* ]]; then
  for n in 2 4 8; do
    timeout -k 10 300 python bench.py --emulate-ranks $n --steps 20 --warmup 3 > "$OUT/${TAG}_emulate_C3_$n.log" 2>&1
    ok_or_stop $? emulate_C3_$n
  done
  timeout -k 10 300 python bench.py --config C4 --emulate-ranks 8 --steps 10 --warmup 2 > "$OUT/${TAG}_emulate_C4_8.log" 2>&1
  ok_or_stop $? emulate_C4_8
fi
if [[ $STEPS == *rehearsal* ]]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 2 --dist-backend gloo --one-device --no-cpu-baseline \
    > "$OUT/${TAG}_rehearsal_2ranks.log" 2>&1
  ok_or_stop $? rehearsal
fi
exit 0
