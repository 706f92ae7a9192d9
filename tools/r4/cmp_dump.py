"""Compare two field_dump.py outputs bitwise: python tools/r4/cmp_dump.py a.pt b.pt"""
import sys
import torch
a, b = torch.load(sys.argv[1], weights_only=True), torch.load(sys.argv[2], weights_only=True)
ok = True
for k in sorted(a):
    same = torch.equal(a[k], b[k])
    ok &= same
    d = "" if same else " max|diff| %.3g" % (a[k].float() - b[k].float()).abs().max().item()
    print("%-28s %s%s" % (k, "identical" if same else "DIFFERENT", d))
print("ALL IDENTICAL" if ok else "SOME DIFFER")
