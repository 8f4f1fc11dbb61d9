#!/bin/bash
# Instruction counts of the single-trace kernel per library build (exp_libs/<name>, "tree" = the
# in-tree library): one rocprofv3 --pmc pass of the bench workload per build, each under its own
# time limit, summarised per bounce by tools/pmc_summary.py.  Usage: bash tools/pmc_ab.sh NAME ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_SMEM"}
for n in "$@"; do
  lib=tree; [ "$n" != tree ] && lib=$ROOT/exp_libs/$n/libwgrt.so
  d=$ROOT/gpurun_out/pmcab_$n/p0
  mkdir -p "$d"
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run --pmc $CTRS -- \
      python3 "$ROOT/tools/with_lib.py" "$lib" "$ROOT/bench.py" --no-cpu-baseline --no-extras --steps 6 --warmup 2 > "$d/log.txt" 2>&1)
  rc=$?
  echo "$n rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_summary.py "$ROOT/gpurun_out/pmcab_$n" > "$ROOT/gpurun_out/pmcab_$n.json" || exit 1
done
exit 0
