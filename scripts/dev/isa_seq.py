"""Condensed instruction sequence of one kernel from an llvm-objdump listing.

    python scripts/dev/isa_seq.py DISASM.txt KERNEL_SUBSTRING [--around mfma] [--n 120]

Keeps the instructions that shape a K loop (MFMA, LDS reads / writes / atomics,
global loads, waitcnts, sleeps, barriers, branches) so the placement of
waits relative to the MFMAs can be read at a glance.  The listing comes from
``hipcc --cuda-device-only -c`` + ``clang-offload-bundler --unbundle`` +
``llvm-objdump -d --no-show-raw-insn``.
"""

import argparse
import re

KEEP = re.compile(r"(v_mfma|ds_read|ds_write|ds_add|buffer_load|global_load|global_atomic|"
                  r"s_waitcnt|s_sleep|s_barrier|s_cbranch|s_branch)")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("listing")
    ap.add_argument("kernel")
    ap.add_argument("--around", default="v_mfma", help="start N lines before the first match")
    ap.add_argument("--before", type=int, default=30)
    ap.add_argument("--n", type=int, default=120)
    a = ap.parse_args(argv)
    lines = open(a.listing).read().split("\n")
    heads = [i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <", l)]
    start = next(i for i in heads if a.kernel in lines[i])
    end = next((i for i in heads if i > start), len(lines))
    seq = [l.strip().split("//")[0].rstrip() for l in lines[start:end]]
    seq = [t for t in seq if KEEP.match(t)]
    first = next((i for i, t in enumerate(seq) if t.startswith(a.around)), 0)
    lo = max(0, first - a.before)
    print("{}: {} kept instructions, {} MFMAs".format(
        lines[start].strip(), len(seq), sum(t.startswith("v_mfma") for t in seq)))
    print("\n".join(seq[lo:lo + a.n]))


if __name__ == "__main__":
    main()
