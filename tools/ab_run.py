"""A/B harness (experiments only): run bench.py against an experiment build of the library
(mli_nerf_amd.build.build(out=...)) built from a modified tree, without the loader's
source-hash check (the tree on disk is the baseline's).  Usage: python tools/ab_run.py <lib.so> [bench args]"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
lib_path = os.path.abspath(sys.argv[1])
from mli_nerf_amd import _lib as L, build as B  # noqa: E402

L.LIB_PATH = lib_path
want = B.built_hash(lib_path)
B.source_hash = lambda: want
import bench  # noqa: E402

bench.main(sys.argv[2:])
