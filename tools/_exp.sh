#!/bin/bash
# scratch experiment driver (one gpurun call): parity of a candidate build, then library A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp; mkdir -p $OUT
set -e
if [ -n "$CAND" ]; then
  cp gpu_ray_tracing_for_waveguide_based_ar_display_amd/libwgrt.so /tmp/libwgrt_orig.so
  cp "$CAND" gpu_ray_tracing_for_waveguide_based_ar_display_amd/libwgrt.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "${TESTK:-fused or replay or golden}" --timeout 200 --timeout-method thread > $OUT/cand_tests.log 2>&1
  cp /tmp/libwgrt_orig.so gpu_ray_tracing_for_waveguide_based_ar_display_amd/libwgrt.so
fi
timeout -k 10 400 python tools/ab_libs.py --rounds 3 --num-iter 20 ${LIBS:-exp_libs/*.so} > $OUT/libs_fused.log 2>&1
timeout -k 10 300 python tools/ab_libs.py --rounds 3 --num-iter 4 ${LIBS:-exp_libs/*.so} > $OUT/libs_single.log 2>&1
if [ -n "$DIAGF" ]; then DIAG_FLAGS="$DIAGF" timeout -k 10 300 python tools/diag.py 1024 7 20 > $OUT/diag_f20.log 2>&1; fi
