"""The ``bench.py --gpus N`` parent on the GPU box (GPU): it counts the GPUs from sysfs and holds
no GPU device file when it spawns the ranks -- after importing torch and counting, /dev/kfd is
not open in a fresh process (a process that initialised HIP must not fork / exec the ranks).
The spawn flow itself runs end to end on CPU in tests/test_bench_launch.py."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r'''
import sys
sys.path.insert(0, %r)
import torch
import bench
n = bench.count_gpus()
held = bench.gpu_handles()
print(n, len(held))
'''


def test_parent_counts_gpus_without_opening_them():
    out = subprocess.run([sys.executable, "-c", PROBE % ROOT], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    n, held = (int(x) for x in out.stdout.split())
    assert n >= 1 and held == 0, out.stdout
