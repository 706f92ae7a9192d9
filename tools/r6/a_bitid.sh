#!/bin/bash
# Stage-a gradient bit-identity of experiment library X against the product (deterministic mode),
# then the stage-a A/B.   X=hrold bash tools/r6/a_bitid.sh
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python tools/r6/grad_a_dump.py /tmp/g_prod.pt || { echo "dump prod failed"; exit 1; }
MLI_HIP_LIB=xlib/$X.so timeout -k 10 200 python tools/r6/grad_a_dump.py /tmp/g_x.pt 2>/dev/null || { echo "dump $X failed"; exit 1; }
python - <<PY || exit 1
import torch
a, b = torch.load("/tmp/g_prod.pt"), torch.load("/tmp/g_x.pt")
print("stage-a grads bit-identical:", {k: bool(torch.equal(a[k], b[k])) for k in a})
PY
bash tools/r6/a_ab.sh
