#!/usr/bin/env python3
"""Static check of the inline-asm MFMAs in a gfx950 assembly listing (hipcc -S).

hipcc pads no hazard for an `asm` statement's operands (guide §5.7 item 2).  The W64 flash forward
(csrc/kernels/flash_attn_fwd.hip) issues its PV MFMAs as inline asm on VGPR A/B operands, so a VALU write
of one of those registers within the two preceding instructions would be read stale.  This walks every
asm MFMA (between ;;#ASMSTART / ;;#ASMEND) and fails when a VALU instruction among the previous
`--window` instructions writes a register of its A or B operand.

    hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only ... -o fwd.s && python tools/check_asm_hazards.py fwd.s
"""
import re
import sys


def regs(tok: str) -> set[int]:
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def main(path: str, window: int = 3) -> int:
    lines = [ln.strip() for ln in open(path)]
    inasm, bad, n = False, [], 0
    recent: list[str] = []  # compiler instructions before the current point
    for k, ln in enumerate(lines):
        if ln.startswith(";;#ASMSTART"):
            inasm = True
            continue
        if ln.startswith(";;#ASMEND"):
            inasm = False
            continue
        if not ln or ln.startswith((";", ".")) or ln.endswith(":"):
            continue
        if inasm and ln.startswith("v_mfma"):
            n += 1
            ops = [t.strip() for t in ln.split(None, 1)[1].split(",")]
            used = regs(ops[1]) | regs(ops[2])
            for prev in recent[-window:]:
                op = prev.split(None, 1)
                if len(op) < 2 or not op[0].startswith("v_") or op[0].startswith("v_mfma"):
                    continue
                dst = regs(op[1].split(",")[0].strip())
                if dst & used:
                    bad.append(f"line {k + 1}: {prev}  ->  {ln}")
        if not inasm:
            recent.append(ln)
    print(f"{n} asm MFMAs checked, {len(bad)} VALU-write -> operand hazards")
    for b in bad[:20]:
        print("  " + b)
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3))
