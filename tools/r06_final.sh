#!/bin/bash
# Round-6 final measurements on the final library: full GPU suite, smoke, fabric-traffic and issue-side PMC
# passes (their own rocprofv3 runs), then the bench line with them (200 steps), the driver's bench command,
# a rocprofv3 kernel-trace summary, the other configs' lines and the 2-rank rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${FINAL_TAG:-r06f}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "[$2] exit $1"; [ "$1" -ne 0 ] && exit "$1"; return 0; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
stop $? pytest; tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
stop $? smoke
cp profiles/traffic.json "$OUT/traffic.json"; cp profiles/pmc.json "$OUT/pmc.json"
timeout -k 10 600 python tools/pmc_traffic.py "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1
stop $? traffic
TAG=${FINAL_TAG:-r06f}/run timeout -k 10 900 bash tools/pmc_passes.sh > "$OUT/pmc.log" 2>&1
stop $? pmc
python tools/pmc_summary.py "$OUT/run_pmc" "$OUT/pmc_summary.json" --merge "$OUT/pmc.json" >> "$OUT/pmc.log" 2>&1
stop $? pmc_summary
timeout -k 10 600 python3 bench.py --steps 200 --warmup 5 --traffic-json "$OUT/traffic.json" --pmc-json "$OUT/pmc.json" \
  > "$OUT/bench_200.jsonl" 2> "$OUT/bench_200.err"
stop $? bench200
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --traffic-json "$OUT/traffic.json" --pmc-json "$OUT/pmc.json" \
  > "$OUT/bench_driver.jsonl" 2> "$OUT/bench_driver.err"
stop $? bench_driver
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
   python3 "$ROOT/bench.py" --no-cpu-baseline --no-extras --steps 200 --warmup 5 > "$OUT/bench_prof.jsonl" 2>&1)
stop $? prof
for c in C2 C4 C5d C5; do
  timeout -k 10 600 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_$c.jsonl" 2> "$OUT/bench_$c.err"
  stop $? bench_$c
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 2 --dist-backend gloo --one-device --no-cpu-baseline \
  > "$OUT/rehearsal_2ranks.log" 2>&1
stop $? rehearsal
exit 0
