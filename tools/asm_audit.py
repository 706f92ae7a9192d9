"""Audit of inline-asm loads in a device assembly file (hipcc -S / -save-temps).  An asm load's
destination counts as written at ;;#ASMEND, so hipcc may copy, spill or reuse it before the data
lands (cdna_hip_programming.md §5.7): flag every compiler instruction that names a destination
register of an asm ds_read / global_load while that load may still be in flight, and every asm
dwordx3/x4 store not followed by s_nop inside its statement.

In flight: each counter keeps its outstanding operations in issue order, the compiler's and the
asm ones alike (vmcnt: global / buffer / scratch loads, stores, atomics and LDS-DMAs, which retire
in issue order; lgkmcnt: LDS operations, and scalar memory loads).  ``s_waitcnt vmcnt(N)`` retires
all but the N youngest vector-memory operations, so only the asm loads older than those are
cleared (clearing every pending load at any count missed a copy made after a wait
that did not yet cover the load).  Scalar loads return out of order: while one is outstanding
an lgkmcnt(N > 0) retires nothing for certain, only lgkmcnt(0) does.  flat_* operations count on
both counters out of order (only a wait to 0 retires them).  Linear scan: control flow is
ignored, so a flagged line is a lead, not a proof.

Usage: python tools/asm_audit.py kernel.s [...]   (exit status 1 on findings)"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
WAIT = re.compile(r"(vmcnt|lgkmcnt)\((\d+)\)")


def regs(text):
    out = set()
    for a, b, c in REG.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def classify(op):
    """The counters an instruction adds an operation to: {'vm', 'lgkm'} subset, and whether the
    lgkm one is a scalar (out-of-order) load."""
    if op.startswith(("global_", "buffer_", "scratch_")):
        return {"vm"}, False
    if op.startswith("flat_"):
        return {"vm", "lgkm"}, False
    if op.startswith("ds_") and op != "ds_nop":
        return {"lgkm"}, False
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_scratch_load")):
        return {"lgkm"}, True
    return set(), False


class Counter:
    """Outstanding operations of one wait counter, oldest first: (asm-load dest regs or None,
    issuing line, out-of-order flag)."""

    def __init__(self):
        self.ops = []

    def issue(self, dest, line, ooo=False):
        self.ops.append((dest, line, ooo))

    def wait(self, n):
        if n == 0:
            self.ops = []
        elif not any(o for _, _, o in self.ops):
            self.ops = self.ops[len(self.ops) - n:] if len(self.ops) > n else self.ops
        # an out-of-order op outstanding: a nonzero count retires nothing for certain

    def pending(self):
        """reg -> line of the asm load that may still be writing it."""
        out = {}
        for dest, line, _ in self.ops:
            if dest:
                for r in dest:
                    out[r] = line
        return out

    def forget(self, regs_):
        self.ops = [(None if d and d & regs_ else d, l, o) for d, l, o in self.ops]


def _apply_waits(text, cnt):
    for kind, n in WAIT.findall(text):
        cnt["vm" if kind == "vmcnt" else "lgkm"].wait(int(n))


def audit(path, out=sys.stdout):
    lines = open(path).read().split("\n")
    cnt = {"vm": Counter(), "lgkm": Counter()}
    issues = 0
    in_asm, block = False, []
    func = "?"

    def note(msg):
        nonlocal issues
        print(msg, file=out)
        issues += 1

    for i, raw in enumerate(lines):
        line = raw.split(";")[0].strip() if not raw.strip().startswith(";;") else raw.strip()
        m = re.match(r"^(_Z\S*):", raw)
        if m:
            func, cnt = m.group(1), {"vm": Counter(), "lgkm": Counter()}
            continue
        if raw.strip() == ";;#ASMSTART":
            in_asm, block = True, []
            continue
        if raw.strip() == ";;#ASMEND":
            in_asm = False
            text = " ".join(block)
            for ins in block:   # in statement order: waits retire what is older
                op = ins.split()[0] if ins.split() else ""
                if op.startswith("s_waitcnt"):
                    _apply_waits(ins, cnt)
                    continue
                kinds, ooo = classify(op)
                dest = None
                if (op.startswith("ds_read") or (op.startswith("global_load") and not op.startswith("global_load_lds"))):
                    dest = regs(ins.split(",")[0])
                for k in kinds:
                    cnt[k].issue(dest, i, ooo)
                if re.match(r"(global|buffer)_store_dwordx[34]", op) and "s_nop" not in text:
                    note("%s:%d %s: asm 16 B store without s_nop in its statement" % (path, i, func[:60]))
            continue
        if in_asm:
            if line:
                block.append(line)
            continue
        if not line or line.startswith(".") or line.endswith(":"):
            continue
        op = line.split()[0]
        if op.startswith("s_waitcnt"):
            _apply_waits(line, cnt)
            continue
        used = regs(line)
        for kind in ("lgkm", "vm"):
            pend = cnt[kind].pending()
            hit = used & set(pend)
            if hit:
                note("%s:%d %s: '%s' names v%s of the asm load at line %d before its %scnt wait" % (
                    path, i + 1, func[:60], line, min(hit), pend[min(hit)] + 1, kind))
                cnt[kind].forget(hit)
        kinds, ooo = classify(op)
        for k in kinds:
            cnt[k].issue(None, i, ooo)
    return issues


if __name__ == "__main__":
    n = sum(audit(p) for p in sys.argv[1:])
    print("asm_audit: %d finding(s)" % n)
    sys.exit(1 if n else 0)
