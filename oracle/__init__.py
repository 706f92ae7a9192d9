"""CPU oracle for the MLI-NeRF stage-b volume-rendering hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``mli_nerf_amd``) may import
this package.  Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` use it, and only as the checker / the timed CPU baseline.

What it is: a plain fp32 PyTorch-on-CPU restatement of the reference algorithm, one
function per reference function, each citing the reference ``file:line`` it restates
(paths relative to the liulisixin/MLI-NeRF checkout).

Pinning:
  * Everything except the hash-grid values is pinned against the reference's own Python
    modules (imported with offline stubs for ``cv2``/``tinycudann``) by the fixtures in
    ``tests/golden/`` and the script ``tests/golden/make_golden.py`` that produced them.
  * The multires hash grid is a restatement of the third-party tiny-cuda-nn ``HashGrid``
    encoding (not vendored, not version-pinned by the reference, absent from this
    container).  Its values are therefore **parity unpinned** against real tiny-cuda-nn;
    the restatement in ``oracle/hashgrid.py`` is the contract both sides implement.
"""
