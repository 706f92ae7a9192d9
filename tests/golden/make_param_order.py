"""Golden fixture: the reference Model's parameter registration order (stage a and b).

The imaginaire optimizer is built over ``model.get_param_groups(cfg.optim)``
(imaginaire/trainers/utils/get_trainer.py:106-118); a torch optimizer state dict indexes its
per-parameter state by position in that list, so a checkpoint's ``optim`` entry
(imaginaire/trainers/base.py:601-607) is only portable if the build lists the parameters in the
reference's order.  This script imports the reference Model with the offline stubs of
make_golden.py (SURVEY.md §8c recipe) and writes the ordered names and shapes to
``param_order.json`` (data only: no reference source travels).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_param_order.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


class _EncodingModule(__import__("torch").nn.Module):
    """tinycudann.Encoding as the tiny-cuda-nn torch bindings define it (restated: a Module
    that registers its flat ``params`` Parameter on itself), so the table takes its place in
    the registration order; the values do not matter here."""

    def __init__(self, n_input_dims, config):
        super().__init__()
        import torch
        from oracle.hashgrid import level_table
        _, total = level_table(config["n_levels"], config["log2_hashmap_size"], config["base_resolution"],
                               config["per_level_scale"])
        self.n_output_dims = config["n_levels"] * config["n_features_per_level"]
        self.params = torch.nn.Parameter(torch.zeros(total * config["n_features_per_level"]))


def main():
    mg.install_stubs()
    sys.modules["tinycudann"].Encoding = _EncodingModule
    from projects.NeuralLumen.model import Model
    out = {}
    for config in ("syn_hotdog_a", "syn_hotdog_b"):
        cfg = mg.reference_cfg(config, 64, 16, 4, 4, 12)
        model = Model(cfg.model, cfg.data)
        groups = model.get_param_groups(cfg.optim)
        ids = {id(p) for p in groups}
        out[config] = dict(
            named=[[n, list(p.shape)] for n, p in model.named_parameters()],
            optimized=[n for n, p in model.named_parameters() if id(p) in ids])
    path = os.path.join(HERE, "param_order.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path)


if __name__ == "__main__":
    main()
