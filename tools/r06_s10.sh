#!/bin/bash
# Round-6 GPU session 10: the full GPU suite on the final library (with the polarisation-selective LUT cases),
# smoke, and the reference's default job through the reference-flow driver.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/r06s10
mkdir -p "$OUT"
export TMPDIR=/tmp WGRT_RESULTS_DIR=$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m gpu_ray_tracing_for_waveguide_based_ar_display_amd.gpu_ray_tracing_pro_fullColor \
  --json "$OUT/main_default_100x75.json" --png "$OUT/Eyebox Center View.png" > "$OUT/main_default_100x75.log" 2>&1
rc=$?; echo "main rc $rc"; tail -12 "$OUT/main_default_100x75.log"; exit $rc
