import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and libgmagg.so")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def golden_manifest():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def golden_case(name):
    for c in golden_manifest()["cases"]:
        if c["name"] == name:
            return c, dict(np.load(os.path.join(GOLDEN, c["file"])))
    raise KeyError(name)


def golden_names(func):
    return [c["name"] for c in golden_manifest()["cases"] if c["func"] == func]


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
