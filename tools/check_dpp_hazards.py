"""Static check of the DPP read-after-write hazard in hand-written inline asm.

gfx950 needs two wait states between a VALU instruction that writes a VGPR and a DPP
instruction that reads that VGPR through its DPP source (src0).  The compiler pads for the DPP
operations it emits itself, but not around inline asm (csrc/lba.hip's v_fmac_f64_dpp /
v_mov_b64_dpp statements): a register copy it inserts in front of one goes unpadded.  This
scans device assembly (hipcc --cuda-device-only -S) and reports every DPP instruction whose src0
registers were written by one of the two preceding VALU instructions with no s_nop in between.

python tools/check_dpp_hazards.py FILE.s [FILE.s ...]   (exit 1 when a hazard is found)
"""
import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def operands(line):
    parts = line.split(None, 1)
    if len(parts) < 2:
        return parts[0], []
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])]
    return parts[0], ops


def scan(path):
    bad = []
    func = "?"
    window = []  # (wait states it provides, written vgprs) of the recent instructions
    for ln, raw in enumerate(open(path), 1):
        line = raw.split(";", 1)[0].strip()
        if not line:
            continue
        if line.endswith(":") and not line.startswith("."):
            if not line.startswith(".L"):
                func = line[:-1]
                window = []
            continue  # a block label: the fall-through path's writes stay in the window
        if line.startswith("."):
            continue
        op, ops = operands(line)
        if op == "s_nop":
            window.append((int(ops[0], 0) + 1 if ops else 1, set()))
        elif op.startswith("v_"):
            if "_dpp" in op and ops:
                src = ops[1] if len(ops) > 1 else ""
                need, got = regs(src), 0
                for states, wr in reversed(window):
                    if got >= 2:
                        break
                    if wr & need:
                        bad.append((path, ln, func, line))
                        break
                    got += states
            wr = regs(ops[0]) if ops and not op.startswith("v_cmp") else set()
            if "permlane" in op and len(ops) > 1:  # the swaps write both operands
                wr |= regs(ops[1])
            window.append((1, wr))
        elif op.startswith("s_") or op.startswith("ds_") or op.startswith("global_") or op.startswith("buffer_"):
            window.append((1, set()))
        window = window[-4:]
    return bad


def main():
    bad = []
    for p in sys.argv[1:]:
        bad += scan(p)
    for path, ln, func, line in bad:
        print(f"{path}:{ln}: {func}: {line}")
    print(f"{len(bad)} DPP read-after-write hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
