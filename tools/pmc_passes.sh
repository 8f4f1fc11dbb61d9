#!/bin/bash
# PMC counter passes over the bench workload's single-trace launches: one counter group per
# rocprofv3 run (--kernel-trace only, no other trace domains), each under its own time limit.
# Output: gpurun_out/<TAG>_pmc/p<i>/ (counter_collection.csv), summarised by tools/pmc_summary.py.
#   PASSES_FILE=file with one counter group per line (default: the built-in list)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-run}
export TMPDIR=/tmp
if [ -n "$PASSES_FILE" ]; then mapfile -t PASSES < "$PASSES_FILE"; else PASSES=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
); fi
i=0
for p in "${PASSES[@]}"; do
  d=$ROOT/gpurun_out/${TAG}_pmc/p$i
  mkdir -p "$d"
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run --pmc $p -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-extras --steps 10 --warmup 2 ${BENCH_ARGS:-} > "$d/log.txt" 2>&1)
  rc=$?
  echo "pass $i rc=$rc: $p"
  if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
