"""Minimal re-statement of imaginaire's config surface (drop-in for the hot path only).

Reference: ``imaginaire/config.py:83-223`` -- YAML files chained by ``_parent_``
(resolved against the repo root), strict recursive merge, and ``--a.b.c=value``
command-line overrides parsed with ``yaml.safe_load``.  Attribute access raises
``AttributeError`` for missing keys so the reference's ``hasattr(cfg, ...)`` feature
switches behave identically.
"""
import copy
import os
import re

import yaml


class _Loader(yaml.SafeLoader):
    """SafeLoader + the float resolver of imaginaire/config.py:109-119 (so ``5e-4`` is a
    float, as in the reference)."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:
     [-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
    |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
    |\.[0-9_]+(?:[eE][-+][0-9]+)?
    |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\.[0-9_]*
    |[-+]?\.(?:inf|Inf|INF)
    |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."))

# README of the reference asks users to replace this placeholder in the YAMLs by hand.
DATASET_FOLDER = os.environ.get("MLI_DATASET_FOLDER", "datasets")


class AttrDict(dict):
    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as exc:
            raise AttributeError(key) from exc

    def __setattr__(self, key, value):
        self[key] = value

    def __deepcopy__(self, memo):
        return AttrDict({k: copy.deepcopy(v, memo) for k, v in self.items()})


def to_attr(obj):
    if isinstance(obj, dict):
        return AttrDict({k: to_attr(v) for k, v in obj.items()})
    if isinstance(obj, list):
        return [to_attr(v) for v in obj]
    return obj


def merge(base, update, strict=False, path=""):
    """config.py:183-198 recursive_update_strict (strict=True refuses unknown keys)."""
    for key, value in update.items():
        if strict and key not in base:
            raise KeyError("unknown config key %s%s" % (path, key))
        if isinstance(value, dict) and isinstance(base.get(key), dict):
            merge(base[key], value, strict, path + key + ".")
        else:
            base[key] = value
    return base


def load_yaml_chain(path, root):
    with open(path) as f:
        text = f.read().replace("{DATASET_FOLDER}", DATASET_FOLDER)
    cfg = yaml.load(text, Loader=_Loader) or {}
    parent = cfg.pop("_parent_", None)
    if parent is None:
        return cfg
    base = load_yaml_chain(os.path.join(root, parent), root)
    return merge(base, cfg)


def parse_overrides(args):
    """config.py:201-223: ``--a.b.c=v`` -> nested dict with yaml-typed values."""
    out = {}
    for arg in args:
        if not arg.startswith("--") or "=" not in arg:
            continue
        key, value = arg[2:].split("=", 1)
        node = out
        parts = key.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = yaml.load(value, Loader=_Loader)
    return out


def load_config(path, root=None, overrides=(), strict_overrides=False):
    root = root or os.getcwd()
    cfg = load_yaml_chain(path, root)
    if overrides:
        merge(cfg, parse_overrides(overrides) if isinstance(overrides, (list, tuple)) else overrides,
              strict=strict_overrides)
    return to_attr(cfg)
