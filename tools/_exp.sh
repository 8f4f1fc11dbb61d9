#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab.py --variants 2,1,3,4,5,6 --rounds 10 > gpurun_out/ab.log 2>&1 || exit $?
timeout -k 10 600 python tools/ab_libs.py --rounds 3 abl/old.so abl/est.so abl/phasor.so > gpurun_out/ab_libs.log 2>&1 || exit $?
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/latency.log 2>&1 || exit $?
echo done
