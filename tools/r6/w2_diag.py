"""Diagnose tests/test_gpu_world2.py: determinism of each form and where overlap != serial."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch  # noqa: E402


def worker(rank, port, results):
    import torch.distributed as dist
    from test_gpu_world2 import _two_steps_b
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        for tag, ov in (("s1", False), ("s2", False), ("o1", True), ("o2", True)):
            results[(rank, tag)] = _two_steps_b(2, ov, 3 + rank)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    from mli_nerf_amd import layout
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    res = ctx.Manager().dict()
    mp.start_processes(worker, args=(port, res), nprocs=2, join=True, start_method="spawn")
    items = layout.trainable_layout("b")[0]
    for a, b in (("s1", "s2"), ("o1", "o2"), ("s1", "o1")):
        for r in range(2):
            x, y = res[(r, a)]["flat"], res[(r, b)]["flat"]
            d = (x != y)
            print(a, b, "rank", r, "differ", int(d.sum()), "max", float((x - y).abs().max()))
            if d.any():
                bad = sorted({name for name, shape, off in items
                              if d[off:off + max(1, int(torch.tensor(shape).prod()))].any()})
                print("   params:", bad[:12])
    print("ranks equal (o1):", torch.equal(res[(0, "o1")]["flat"], res[(1, "o1")]["flat"]),
          "(s1):", torch.equal(res[(0, "s1")]["flat"], res[(1, "s1")]["flat"]))
