#!/usr/bin/env python3
"""Static check of the inline-asm MFMAs in a gfx950 assembly listing (hipcc -S).

hipcc pads no hazard for an `asm` statement's operands (guide §5.7 item 2).  The W64 flash forward
(csrc/kernels/flash_attn_fwd.hip) issues its PV MFMAs as inline asm on VGPR A/B operands, so a VALU write
of one of those registers within the two preceding instructions would be read stale.  This walks every
asm MFMA (between ;;#ASMSTART / ;;#ASMEND) and fails when a VALU instruction among the previous
`--window` instructions writes a register of its A or B operand (RAW), and when any compiler instruction
touches an accumulator register of the kernel-owned range (`owned` and up: the W64 forward's O).  Writes of
an A / B register right AFTER an MFMA (WAR) are listed for information only: the hardware reads A / B at
issue, and hipcc emits the same pattern after its own builtin MFMAs.

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


def regs_in(text: str) -> set[int]:
    """Every VGPR named in an operand list."""
    out = set()
    for lo, hi in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        out |= set(range(int(lo), int(hi) + 1))
    for r in re.findall(r"\bv(\d+)\b", text):
        out.add(int(r))
    return out


def agprs(text: str) -> set[int]:
    out = set()
    for lo, hi in re.findall(r"\ba\[(\d+):(\d+)\]", text):
        out |= set(range(int(lo), int(hi) + 1))
    for r in re.findall(r"\ba(\d+)\b", text):
        out.add(int(r))
    return out


def main(path: str, window: int = 3, owned: int = 128) -> int:
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
    # WAR pass: instructions after each asm MFMA (compiler or asm) that write its A / B registers
    war = []
    flat = [(k, ln) for k, ln in enumerate(lines) if ln and not ln.startswith((";", ".")) and not ln.endswith(":")]
    for idx, (k, ln) in enumerate(flat):
        if ln.startswith("v_mfma") and "a[" in ln.split(",")[0]:
            ops = [t.strip() for t in ln.split(None, 1)[1].split(",")]
            used = regs(ops[1]) | regs(ops[2])
            for k2, nxt in flat[idx + 1: idx + 1 + 2 * window]:
                op = nxt.split(None, 1)
                if len(op) < 2 or op[0].startswith(("s_", "v_mfma", "buffer_", "global_store", "ds_write")):
                    continue
                dst = regs(op[1].split(",")[0].strip())
                if dst & used:
                    war.append(f"line {k2 + 1}: {nxt}  after  line {k + 1}: {ln}")
    # asm MFMA with a VGPR destination (the W64 S MFMAs): no instruction may read or write that destination
    # within 12 wait states (8-pass XDL result latency; an s_nop N counts N + 1), except the next MFMA of
    # the same accumulation chain taking it whole as SrcC
    dres = []
    for idx, (k, ln) in enumerate(flat):
        if not (ln.startswith("v_mfma") and ln.split(None, 1)[1].split(",")[0].strip().startswith("v")):
            continue
        ops = [t.strip() for t in ln.split(None, 1)[1].split(",")]
        dst = regs(ops[0])
        states = 0
        for k2, nxt in flat[idx + 1:]:
            if states >= 12:
                break
            op = nxt.split(None, 1)
            if op[0].startswith("v_mfma") and len(op) > 1:
                o2 = [t.strip() for t in op[1].split(",")]
                if regs(o2[0]) == dst and regs(o2[3]) == dst:
                    break  # the chain continues: its own hazard is checked at that MFMA
            if len(op) > 1 and op[0] != "s_nop" and (regs_in(op[1]) & dst):
                dres.append(f"line {k2 + 1}: {nxt}  {states} states after  line {k + 1}: {ln}")
                break
            states += int(op[1]) + 1 if op[0] == "s_nop" else 1
    print(f"VGPR-destination asm MFMAs: result read / overwritten within 12 wait states: {len(dres)}")
    for d in dres[:10]:
        print("  " + d)
    bad += dres
    # ownership: accumulator registers >= `owned` belong to the kernel's asm; the compiler must not touch them
    inasm, own, comp_agpr = False, [], 0
    for k, ln in enumerate(lines):
        if ln.startswith(";;#ASMSTART"):
            inasm = True
        elif ln.startswith(";;#ASMEND"):
            inasm = False
        elif not inasm and ln and not ln.startswith((";", ".")) and not ln.endswith(":"):
            regs_a = agprs(ln.split(";")[0])
            if regs_a:
                comp_agpr += 1
                if max(regs_a) >= owned:
                    own.append(f"line {k + 1}: {ln}")
    print(f"compiler instructions touching accumulator registers: {comp_agpr}; inside the owned range a[{owned}:]: {len(own)}")
    for o in own[:10]:
        print("  " + o)
    bad += own
    # M0: a function whose asm owns M0 (the "m0-owned" LDS-DMA pieces set it without saving it) must have no
    # compiler instruction that reads or writes M0
    m0bad, fn, owns, uses = [], None, False, []
    for k, ln in enumerate(lines + ["_Zend:"]):
        if re.match(r"^_Z\S*:", ln) or ln.startswith(".Lfunc_end"):
            if owns and uses:
                m0bad += [f"{fn}: {u}" for u in uses]
            fn, owns, uses, inasm = ln, False, [], False
            continue
        if ln.startswith(";;#ASMSTART"):
            inasm = True
        elif ln.startswith(";;#ASMEND"):
            inasm = False
        elif inasm and "m0-owned" in ln:
            owns = True
        elif not inasm and ln and not ln.startswith((";", ".")) and re.search(r"\bm0\b", ln.split(";")[0]):
            uses.append(f"line {k + 1}: {ln}")
    print(f"compiler M0 uses in functions whose asm owns M0: {len(m0bad)}")
    for o in m0bad[:10]:
        print("  " + o)
    bad += m0bad
    print(f"{n} asm MFMAs checked, {len(bad)} write -> operand (RAW) hazards ({len(war)} WAR reuses, informational)")
    for b in bad[:20]:
        print("  " + b)
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3,
                  int(sys.argv[3]) if len(sys.argv) > 3 else 128))
