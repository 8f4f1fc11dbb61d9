#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run, --kernel-trace only, no
# sys/runtime trace) over tools/ab.py for the given variants.  Output: gpurun_out/pmc/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-1 2}
ABARGS=${ABARGS:-}
PASSES=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F32 SQ_INST_LEVEL_VMEM"
)
for v in $VARIANTS; do
  i=0
  for p in "${PASSES[@]}"; do
    d=$ROOT/gpurun_out/pmc/v${v}_p$i
    mkdir -p "$d"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run --pmc $p -- \
        python3 "$ROOT/tools/ab.py" --variants $v --rounds 2 $ABARGS > "$d/log.txt" 2>&1)
    rc=$?
    echo "variant $v pass $i rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    i=$((i+1))
  done
done
