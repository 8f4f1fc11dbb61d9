#!/usr/bin/env python3
"""One line per variant from tools/pmc_summary.py output (normalised per bounce)."""
import json
import subprocess
import sys

d = json.loads(subprocess.run([sys.executable, "tools/pmc_summary.py"], capture_output=True, text=True).stdout)
b = float(sys.argv[1]) if len(sys.argv) > 1 else 8641973
for v, c in d.items():
    g = lambda k: c.get(k, float("nan"))
    print(v, "VALU/b %.1f SALU/b %.1f lane-util %.3f VMEMrd/b %.2f F64fma/b %.1f F64trans/b %.2f wait_inst %.2f "
          "wait_any %.2f fetchKB %.0f writeKB %.0f L2hit %.3f waves %d" % (
              g("SQ_INSTS_VALU") / b, g("SQ_INSTS_SALU") / b,
              g("SQ_THREAD_CYCLES_VALU") / (g("SQ_ACTIVE_INST_VALU") * 64), g("SQ_INSTS_VMEM_RD") / b,
              g("SQ_INSTS_VALU_FMA_F64") / b, g("SQ_INSTS_VALU_TRANS_F64") / b,
              g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"), g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
              g("FETCH_SIZE"), g("WRITE_SIZE"), g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")),
              g("SQ_WAVES")))
