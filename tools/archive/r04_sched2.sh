#!/bin/bash
# Round-4: the scheduler-strategy builds on the latency-bound launches (C2, C3 shards of 8 / 4 / 2 ranks).
# (exp_libs as in tools/r04_sched.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${CASES:-C2:1 C3:8 C3:4 C3:2}; do
  c=${spec%%:*}; n=${spec##*:}
  timeout -k 10 500 python tools/ab.py tree ${NAMES:-silp sitilp} --rounds ${ROUNDS:-5} --config $c --shard $n --fused 2 > gpurun_out/r04_ab_sched_${c}_s$n.log 2>&1
  rc=$?; echo "ab $c shard $n rc $rc"; grep SUMMARY gpurun_out/r04_ab_sched_${c}_s$n.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/r04_ab_sched_${c}_s$n.log; exit $rc; fi
done
