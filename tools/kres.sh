#!/bin/bash
# Register / scratch / occupancy summary of the kernels of one build of wgrt_trace.hip
# (hipcc -Rpass-analysis=kernel-resource-usage).  Extra hipcc flags (e.g. -DWGRT_EDGE_NOINLINE) pass through.
#   tools/kres.sh [-Dmacro ...]
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-fast-math -mllvm -disable-machine-licm --offload-arch=gfx950 \
  --cuda-device-only -c -Rpass-analysis=kernel-resource-usage -I include "$@" -o /tmp/kres.o \
  gpu_ray_tracing_for_waveguide_based_ar_display_amd/csrc/wgrt_trace.hip 2>&1 |
  sed -n 's/.*remark: *\(.*\) \[-Rpass-analysis=kernel-resource-usage\]/\1/p' |
  awk '/^Function Name:/ {n=$3; sub(/^_ZN12_GLOBAL__N_1[0-9]+/, "", n); sub(/EvN4wgrt9TraceArgs.*/, "", n); sub(/EvN4wgrt.*/, "", n)}
       /^TotalSGPRs:/ {s=$2} /^VGPRs:/ {v=$2} /^ScratchSize/ {sc=$3}
       /^Occupancy/ {o=$3} /^SGPRs Spill:/ {ss=$3} /^VGPRs Spill:/ {vs=$3; print n, "vgpr=" v, "sgpr=" s, "scratch=" sc, "occ=" o, "spill=" ss "/" vs}'
