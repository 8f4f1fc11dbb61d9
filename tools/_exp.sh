#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "7 or 8 or 9 or forced or rare or invariance or edge" > gpurun_out/pytest_exp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_exp.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/ab.py --variants 5,7 --rounds 8 > gpurun_out/ab.log 2>&1 || exit $?
timeout -k 10 200 python tools/phases.py 7 > gpurun_out/phases7.log 2>&1 || exit $?
