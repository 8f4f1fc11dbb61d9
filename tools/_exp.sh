#!/bin/bash
# scratch experiment script (GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab.py --variants 2,4,5,6,3 --rounds 10 > gpurun_out/ab64.log 2>&1 || exit $?
WGRT_CELL_MM=0.03125 timeout -k 10 300 python tools/ab.py --variants 2,4,5,6 --rounds 10 > gpurun_out/ab32.log 2>&1 || exit $?
WGRT_CELL_MM=0.0078125 timeout -k 10 300 python tools/ab.py --variants 2,4,5,6 --rounds 10 > gpurun_out/ab128.log 2>&1 || exit $?
echo done
