#!/bin/bash
# scratch experiment driver (one gpurun call)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp; mkdir -p $OUT
set -e
timeout -k 10 200 python tools/ab.py --variants 7f,7f,7f,7f,7f --workgroups 768,640,512,384,1024 --num-iter 4 --rounds 6 > $OUT/wg4.log 2>&1
timeout -k 10 200 python tools/ab.py --variants 7,7,7,7 --workgroups 768,640,512,384 --num-iter 1 --rounds 6 > $OUT/wg1.log 2>&1
WGRT_JMAX_HOPS=2 timeout -k 10 200 python tools/ab.py --variants 7f,7 --num-iter 4 --rounds 6 > $OUT/hops2.log 2>&1
WGRT_JMAX_HOPS=4 timeout -k 10 200 python tools/ab.py --variants 7f,7 --num-iter 4 --rounds 6 > $OUT/hops4.log 2>&1
timeout -k 10 200 python tools/ab.py --variants 7f,7 --num-iter 16 --rounds 4 > $OUT/it16.log 2>&1
timeout -k 10 200 python tools/ab.py --variants 7f,7 --num-iter 4 --rounds 4 --R 4096 > $OUT/r4096.log 2>&1
