"""Nested dict <-> .npz (no pickle) for the committed golden fixtures in tests/golden/.

Keys are '/'-joined paths; 0-d arrays come back as Python scalars. Loaded with numpy's default
allow_pickle=False."""
import numpy as np


def _flatten(prefix, obj, out):
    if isinstance(obj, dict):
        for k, v in obj.items():
            _flatten(f"{prefix}/{k}" if prefix else str(k), v, out)
    elif isinstance(obj, (list, tuple)) and obj and isinstance(obj[0], dict):
        for i, v in enumerate(obj):
            _flatten(f"{prefix}/#{i}", v, out)
    else:
        out[prefix] = np.asarray(obj)


def save(path, obj):
    flat = {}
    _flatten("", obj, flat)
    np.savez_compressed(path, **flat)


def load(path):
    root = {}
    with np.load(path) as z:
        for key in z.files:
            a = z[key]
            v = a.item() if a.ndim == 0 else a
            parts = key.split("/")
            node = root
            for p in parts[:-1]:
                node = node.setdefault(p, {})
            node[parts[-1]] = v
    return _lists(root)


def _lists(node):
    if not isinstance(node, dict):
        return node
    node = {k: _lists(v) for k, v in node.items()}
    if node and all(k.startswith("#") for k in node):
        return [node[f"#{i}"] for i in range(len(node))]
    return node
