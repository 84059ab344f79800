#!/usr/bin/env python3
"""Check the gfx950 ISA of the kernels for hand-placed asynchronous loads into registers.

Round 3's `row_policy_head` (kernels.hip) issued the step-counter load as inline asm with a VGPR
output and waited for it (`s_waitcnt vmcnt(0)`) only where the Philox noise is drawn (round 4: an
ordinary divergent load the compiler tracks; `asm_vgpr_loads` must find none).  The compiler treats the
asm output as defined at the asm statement, so it is free to copy or spill that register before the
wait; the copy then reads a value that has not landed, and the late load overwrites whatever the
register was reused for (a round-3 experiment with 256-VGPR heads faulted on Humanoid this way).
This check fails when any instruction between such a load and the next `vmcnt(0)` wait touches
the load's destination registers.

    python3 tools/asm_hazard.py kernels.s          # exit 1 and a report on a hazard
"""
from __future__ import annotations

import re
import sys

_RANGE = re.compile(r"\bv\[(\d+):(\d+)\]")
_SINGLE = re.compile(r"\bv(\d+)\b")
_LOAD = re.compile(r"global_load_dword\w*\s+(v\[\d+:\d+\]|v\d+)")
# a load with a register destination (the LDS-DMA forms, global_load_lds_*, write LDS only)
_VGPR_LOAD = re.compile(r"\b(global|buffer|flat)_load_(?!lds)\w+\s+(v\[\d+:\d+\]|v\d+)")


def asm_vgpr_loads(asm: str) -> list[str]:
    """Loads into registers issued from inline asm (the compiler cannot track their waits)."""
    out, func, in_asm = [], "?", False
    for i, line in enumerate(asm.split("\n")):
        s = line.strip()
        m = re.match(r"^(_Z\S+):", s)
        if m:
            func = m.group(1)
        if s.startswith(";;#ASMSTART"):
            in_asm = True
        elif s.startswith(";;#ASMEND"):
            in_asm = False
        elif in_asm and _VGPR_LOAD.search(s.split(";")[0]):
            out.append(f"{func}: line {i + 1}: {s}")
    return out


def _regs(text: str) -> set[int]:
    out = set()
    for a, b in _RANGE.findall(text):
        out.update(range(int(a), int(b) + 1))
    for a in _SINGLE.findall(_RANGE.sub("", text)):
        out.add(int(a))
    return out


def scan(asm: str) -> list[str]:
    """Hazards in every function of `asm` (the text of a `-S` device compile)."""
    problems = []
    func = "?"
    lines = asm.split("\n")
    in_asm = False
    block: list[int] = []
    for i, line in enumerate(lines):
        s = line.strip()
        m = re.match(r"^(_Z\S+):", s)
        if m:
            func = m.group(1)
        if s.startswith(";;#ASMSTART"):
            in_asm, block = True, []
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            text = "\n".join(lines[j] for j in block)
            lm = _LOAD.search(text)
            if lm and "vmcnt(0)" not in text:
                dst = _regs(lm.group(1))
                for j in range(i + 1, len(lines)):
                    t = lines[j].split(";")[0]
                    if "s_waitcnt" in t and "vmcnt(0)" in t:
                        break
                    if re.match(r"^\s*\.Lfunc_end", lines[j]):
                        break
                    if t.strip() and _regs(t) & dst:
                        problems.append(f"{func}: line {j + 1}: '{t.strip()}' touches {sorted(dst)} "
                                        f"before the asm load (line {i}) is waited for")
                        break
            continue
        if in_asm:
            block.append(i)
    return problems


def main(argv):
    if len(argv) != 2:
        print(__doc__)
        return 2
    with open(argv[1]) as f:
        text = f.read()
    probs = scan(text) + asm_vgpr_loads(text)
    for p in probs:
        print(p)
    return 1 if probs else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
