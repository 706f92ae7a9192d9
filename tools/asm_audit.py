"""Audit of inline-asm loads in a device assembly file (hipcc --cuda-device-only -S).  An asm
load's destination counts as written at ;;#ASMEND, so hipcc may copy, spill or reuse it before
the data lands (cdna_hip_programming.md §5.7): flag every compiler instruction that names a
destination register of an asm ds_read / global_load before the next s_waitcnt of that counter
(lgkmcnt / vmcnt; asm or compiler), and every asm dwordx3/x4 store not followed by s_nop inside
its statement.  Linear scan (control flow ignored: a flagged line is a lead, not a proof).
Usage: python tools/asm_audit.py kernel.s [...]"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for a, b, c in REG.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def audit(path):
    lines = open(path).read().split("\n")
    pending = {"lgkm": {}, "vm": {}}  # reg -> line of the asm load
    issues = 0
    in_asm, block = False, []
    func = "?"
    for i, raw in enumerate(lines):
        line = raw.split(";")[0].strip() if not raw.strip().startswith(";;") else raw.strip()
        m = re.match(r"^(_Z\S*):", raw)
        if m:
            func, pending = m.group(1), {"lgkm": {}, "vm": {}}
            continue
        if raw.strip() == ";;#ASMSTART":
            in_asm, block = True, []
            continue
        if raw.strip() == ";;#ASMEND":
            in_asm = False
            text = " ".join(block)
            for ins in block:
                if "s_waitcnt" in ins:
                    if "lgkmcnt" in ins:
                        pending["lgkm"].clear()
                    if "vmcnt" in ins:
                        pending["vm"].clear()
            for ins in block:
                op = ins.split()[0] if ins.split() else ""
                if op.startswith("ds_read"):
                    for r in regs(ins.split(",")[0]):
                        pending["lgkm"][r] = i
                elif op.startswith("global_load") and not op.startswith("global_load_lds"):
                    for r in regs(ins.split(",")[0]):
                        pending["vm"][r] = i
                if re.match(r"(global|buffer)_store_dwordx[34]", op) and "s_nop" not in text:
                    print("%s:%d %s: asm 16 B store without s_nop in its statement" % (path, i, func[:60]))
                    issues += 1
            continue
        if in_asm:
            if line:
                block.append(line)
            continue
        if not line or line.startswith(".") or line.endswith(":"):
            continue
        if line.startswith("s_waitcnt"):
            if "lgkmcnt" in line:
                pending["lgkm"].clear()
            if "vmcnt" in line:
                pending["vm"].clear()
            continue
        used = regs(line)
        for kind in ("lgkm", "vm"):
            hit = used & set(pending[kind])
            if hit:
                print("%s:%d %s: '%s' names v%s of the asm load at line %d before its %scnt wait" % (
                    path, i + 1, func[:60], line, min(hit), pending[kind][min(hit)] + 1, kind))
                issues += 1
                for r in hit:
                    pending[kind].pop(r, None)
    return issues


if __name__ == "__main__":
    n = sum(audit(p) for p in sys.argv[1:])
    print("asm_audit: %d finding(s)" % n)
    sys.exit(1 if n else 0)
