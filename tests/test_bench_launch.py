"""``bench.py --gpus N`` end to end on CPU (the driver's multi-GPU run goes through this path).

The parent counts GPUs from sysfs (never initialising HIP), refuses to spawn while it holds a GPU
device file, and starts N ranks with torch.distributed.run's environment; each rank runs the real
``bench.main()`` -- argument parsing, the trainer / inference flow, the barrier + max-over-ranks
timing and rank 0's one JSON line.  On CPU the ranks swap in ``bench.PLATFORM``'s CPU stand-in,
gloo collectives, tests/stub_engine.py for the render kernels and a host ray feed for
``mli_ray_batch`` (test infrastructure only; the product bench runs ``HipPlatform``)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))

_RANK = r'''
import sys
sys.path.insert(0, ROOT_DIR)
sys.path.insert(0, TESTS_DIR)
import torch
import bench
import stub_engine
from mli_nerf_amd import data as D, synthetic


class CpuPlatform(bench.HipPlatform):
    name = "cpu-stub"

    def device(self, local):
        return torch.device("cpu")

    def sync(self):
        pass

    def priority_range(self):
        return (0, 0)

    def backend(self, rehearse):
        return "gloo"


class HostFeed:
    """mli_ray_batch stand-in: the reference's host draw (randperm) on the synthetic frames."""

    def __init__(self, device=None, images=None, pseudo=None, cameras=None):
        self.images, self.pseudo, self.cameras = images, pseudo, cameras

    def batch(self, idx, seed, R, stream=None):
        g = torch.Generator().manual_seed(int(seed) & 0x7FFFFFFF)
        ray_idx = torch.randperm(self.images.shape[-1], generator=g)[:R]
        intr, pose, light = self.cameras[idx % len(self.cameras)]
        ref, sha, cert = self.pseudo
        return dict(idx=torch.tensor([idx]), ray_idx=ray_idx[None], image_sampled=self.images[idx][:, ray_idx].t()[None],
                    intr=intr[None], pose=pose[None], pose_light=light[None],
                    pseudo_ref_sampled=ref[idx][:, ray_idx].t()[None], pseudo_sha_sampled=sha[idx][ray_idx][None, :, None],
                    pseudo_visibility_certainty_sampled=cert[idx][ray_idx][None, :, None])


bench.PLATFORM = CpuPlatform()
stub_engine.install()
stub_engine.install_cpu_streams()
D.DeviceFeed = HostFeed
# a 2^12 hash table on CPU (the bench builds the full 2^22 one)
from mli_nerf_amd import configs
_sd, _preset = synthetic.make_state_dict, configs.preset
synthetic.make_state_dict = lambda log2T=12, **kw: _sd(log2T=12, **kw)
configs.preset = lambda name, **kw: _preset(name, **dict(kw, log2T=12))
bench.main(sys.argv[1:])
'''


def test_count_gpus_from_sysfs(tmp_path, monkeypatch):
    import bench
    nodes = tmp_path / "nodes"
    for i, simd in enumerate((0, 256, 256, 256)):    # node 0: the CPU (no SIMDs)
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("cpu_cores_count %d\nsimd_count %d\nmax_waves_per_simd 8\n" % (8 * (simd == 0), simd))
    real = os.path.isdir
    monkeypatch.setattr(bench.os.path, "isdir", lambda p: True if p == "/sys/class/kfd/kfd/topology/nodes" else real(p))
    real_listdir, real_open = os.listdir, open

    def listdir(p):
        return real_listdir(str(nodes)) if p == "/sys/class/kfd/kfd/topology/nodes" else real_listdir(p)

    def fake_open(p, *a, **k):
        if str(p).startswith("/sys/class/kfd/kfd/topology/nodes/"):
            p = str(nodes / os.path.relpath(p, "/sys/class/kfd/kfd/topology/nodes"))
        return real_open(p, *a, **k)
    monkeypatch.setattr(bench.os, "listdir", listdir)
    monkeypatch.setattr("builtins.open", fake_open)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.count_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert bench.count_gpus() == 2


def test_launcher_refuses_while_holding_a_gpu_file(monkeypatch):
    import bench
    assert bench.gpu_handles() == []          # this CPU process: no /dev/kfd
    monkeypatch.setattr(bench, "gpu_handles", lambda: ["/dev/kfd"])
    with pytest.raises(RuntimeError):
        bench.launch_workers(2, ["--steps", "1"], script=os.path.join(ROOT, "bench.py"))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["train", "infer"])
def test_bench_main_gpus2_end_to_end(mode, tmp_path, capfd, monkeypatch):
    """bench.main(['--gpus', '2', ...]) in this (GPU-free) process: two ranks, one JSON line from
    rank 0 with n_gpus 2 and the max-over-ranks time, exit code 0."""
    import bench
    rank_py = tmp_path / "rank.py"
    rank_py.write_text(_RANK.replace("ROOT_DIR", repr(ROOT)).replace("TESTS_DIR", repr(TESTS)))
    monkeypatch.setattr(bench, "WORKER_SCRIPT", str(rank_py))
    monkeypatch.setattr(bench, "count_gpus", lambda: 2)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    argv = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-kernel-timing"]
    if mode == "train":
        argv += ["--rays", "32", "--pipeline", "off", "--tail", "three"]   # the stub stands in for the three-call tail
    else:
        argv += ["--mode", "infer", "--size", "8", "--chunk", "16", "--frames", "2"]
    with pytest.raises(SystemExit) as ex:
        bench.main(argv)
    assert ex.value.code == 0
    assert bench.gpu_handles() == []          # the parent never opened the GPU
    lines = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, lines             # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["value"] > 0
    if mode == "train":
        assert rec["config"]["global_rays"] == 64 and rec["config"]["parallelism"] == "dp2"
        assert rec["scaling"] == "weak"
    else:
        assert rec["config"]["parallelism"] == "tiles2" and rec["scaling"] == "strong"
