#!/bin/bash
# The single-trace grid rule (wgrt_launch_opts.grid_sqrt_k, default 6.5) on the deep / balanced LUT profiles:
# tools/ab.py of K = 4.5 / 6.5 / 9 / resident grid on C2 and on rank 0's quarter and eighth shards of C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
TAG=${TAG:-r04grid}
mkdir -p "$OUT"
export TMPDIR=/tmp
NAMES="tree tree+grid_sqrt_k=4.5 tree+grid_sqrt_k=9.0 tree+grid_sqrt_k=-1.0"
for prof in ${PROFILES:-deep balanced default}; do
  for spec in "C2 1" "C3 4" "C3 8"; do
    set -- $spec
    timeout -k 10 300 python tools/ab.py $NAMES --rounds ${ROUNDS:-2} --config $1 --shard $2 --profile $prof \
      --launches 10 --fused 4 > "$OUT/${TAG}_${prof}_$1_s$2.log" 2>&1
    rc=$?; echo "$prof $1 shard $2 rc $rc"; grep SUMMARY "$OUT/${TAG}_${prof}_$1_s$2.log"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/${TAG}_${prof}_$1_s$2.log"; exit $rc; fi
  done
done
exit 0
