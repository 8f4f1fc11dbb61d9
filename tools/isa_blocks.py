"""Per-basic-block instruction census of one kernel in a device assembly listing.

  hipcc ... --cuda-device-only -S -gline-tables-only -o trace.s csrc/wgrt_trace.hip
  python tools/isa_blocks.py trace.s 'trace_jones_kernelIjLb0ELb0E' [--listing]

For every block: instruction count, VALU / SALU / VMEM / SMEM / LDS / branch split, loop depth,
the source lines (file:line) most of its instructions come from, and its branch targets.  A
static census: which blocks run how often is the reader's judgement (or a PMC pass's).
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "br"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache", "s_memtime", "s_memrealtime")):
        return "smem"
    if op.startswith("s_waitcnt") or op.startswith(("s_nop", "s_barrier", "s_sleep", "s_setprio")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    listing = "--listing" in sys.argv
    files, lines, inside, blocks, cur = {}, open(path).read().splitlines(), False, [], None
    loc = "?"
    for ln in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', ln)
        if m:
            files[m.group(1)] = m.group(2).rsplit("/", 1)[-1]
            continue
        if not inside:
            if re.match(r'^_Z\S*' + re.escape(name) + r'\S*:', ln):
                inside = True
                cur = {"label": "entry", "ins": [], "loop": 0}
            continue
        if ln.startswith(".Lfunc_end"):
            blocks.append(cur)
            break
        m = re.match(r'^(\.LBB\w+|; %bb\.\d+):?\s*(?:;.*Depth=(\d+))?', ln)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "ins": [], "loop": int(m.group(2) or 0)}
            continue
        m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', ln)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))[:10]}:{m.group(2)}"
            continue
        s = ln.strip()
        if not s or s.startswith((".", ";")):
            continue
        op = s.split()[0]
        cur["ins"].append((op, classify(op), loc, s))
    tot = Counter()
    for b in blocks:
        c = Counter(k for _, k, _, _ in b["ins"])
        if b["loop"]:
            tot.update(c)
        srcs = Counter(l for _, _, l, _ in b["ins"]).most_common(4)
        tg = [s.split()[-1].replace(".LBB", "") for op, k, _, s in b["ins"] if k == "br"]
        print(f"{b['label']:<10} d{b['loop']} n={len(b['ins']):4d} v={c['valu']:3d} s={c['salu']:3d} "
              f"m={c['vmem']:2d} sm={c['smem']:2d} ds={c['lds']:2d} br={c['br']:2d} | "
              + ", ".join(f"{l}x{n}" for l, n in srcs) + " | " + " ".join(tg))
        if listing:
            for op, k, l, s in b["ins"]:
                print(f"      {s:<70} {l}")
    print("loop blocks total:", dict(tot))


if __name__ == "__main__":
    main()
