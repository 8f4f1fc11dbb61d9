#!/bin/bash
# Iteration loop on the GPU box: parity tests, interleaved A/B, PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -rf gpurun_out/pmc
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab.py ${AB_ARGS:---variants 1,2} > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
if [ -z "$NO_PMC" ]; then bash tools/pmc.sh > gpurun_out/pmc.log 2>&1; echo "pmc rc=$?"; fi
