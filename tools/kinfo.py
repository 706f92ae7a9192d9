"""Per-kernel summary of a device assembly file (hipcc --cuda-device-only -S): scratch accesses,
MFMAs, barriers and every s_waitcnt the COMPILER inserted (inline-asm waits are skipped) -- the
check for compiler vmcnt(0) drains behind LDS-DMAs / stores.
Usage: python tools/kinfo.py kernel.s [name-substring]"""
import re
import sys


def main(path, pat="_kernel"):
    s = open(path).read().split("\n")
    names = [(i, l.split(":")[0]) for i, l in enumerate(s) if re.match(r"^_Z\S*%s\S*:" % pat, l)]
    for i, n in names:
        j = i
        while not s[j].strip().startswith(".size"):
            j += 1
        body = s[i:j]
        asm, waits = False, {}
        for line in body:
            if "ASMSTART" in line:
                asm = True
                continue
            if "ASMEND" in line:
                asm = False
                continue
            if not asm and "s_waitcnt" in line:
                waits[line.strip()] = waits.get(line.strip(), 0) + 1
        print(n, "scratch", sum("scratch_" in x for x in body), "mfma", sum("v_mfma" in x for x in body),
              "barrier", sum("s_barrier" in x for x in body),
              {k: v for k, v in sorted(waits.items()) if "vmcnt" in k})


if __name__ == "__main__":
    main(*sys.argv[1:])
