#!/bin/bash
# One A/B GPU session: parity tests of the tree's library, then tools/ab.py over exp_libs builds and
# one instruction-count PMC pass of the tree's library.   NAMES="base adv"  TAG=r03d  TESTS=...  PARITY="adv"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
TAG=${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 "$OUT/${TAG}_pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
# PARITY="name ...": the same tests on exp_libs builds (tools/with_lib.py)
for v in $PARITY; do
  timeout -k 10 600 python -u tools/with_lib.py $(pwd)/exp_libs/$v/libwgrt.so -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 240 \
    --timeout-method thread > "$OUT/${TAG}_pytest_$v.log" 2>&1
  rc=$?; echo "pytest $v rc $rc"; tail -2 "$OUT/${TAG}_pytest_$v.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 400 python tools/ab.py ${NAMES:-base adv} --rounds ${ROUNDS:-4} --config C3 > "$OUT/${TAG}_ab_C3.log" 2>&1 || exit $?
grep SUMMARY "$OUT/${TAG}_ab_C3.log"
if [ -n "$C5" ]; then
  timeout -k 10 300 python tools/ab.py ${NAMES:-base adv} --rounds 1 --config C5 --launches 2 --fused 2 > "$OUT/${TAG}_ab_C5.log" 2>&1 || exit $?
  grep SUMMARY "$OUT/${TAG}_ab_C5.log"
fi
d=$OUT/${TAG}_pmc_insts
mkdir -p "$d"
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
   --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS -- \
   python3 "$OLDPWD/bench.py" --no-cpu-baseline --no-extras --steps 10 --warmup 2 > "$d/log.txt" 2>&1)
echo "pmc rc $?"
exit 0
