#!/bin/bash
# Round-4 A/B of the AMDGPU machine scheduler strategy (exp_libs built by tools/ab_build.py with
# -mllvm -amdgpu-sched-strategy=...) against the tree's library, on C3, C2 and C4.
# (The exp_libs builds: python tools/ab_build.py silp=-mllvm,-amdgpu-sched-strategy=max-ilp
#  smem=-mllvm,-amdgpu-sched-strategy=max-memory-clause sitilp=-mllvm,-amdgpu-sched-strategy=iterative-ilp)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-C3 C2 C4}; do
  timeout -k 10 500 python tools/ab.py tree ${NAMES:-silp smem sitilp} --rounds 3 --config $c --fused 10 > gpurun_out/r04_ab_sched_$c.log 2>&1
  rc=$?; echo "ab $c rc $rc"; grep SUMMARY gpurun_out/r04_ab_sched_$c.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/r04_ab_sched_$c.log; exit $rc; fi
done
