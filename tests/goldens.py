"""Helpers to read the golden fixtures written by oracle/make_goldens.py."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))  # allow_pickle=False (default)
    d = {k: z[k] for k in z.files}
    cfg = json.loads(str(d.pop("cfg"))) if "cfg" in d else None
    return cfg, d


def section(d, prefix):
    n = len(prefix) + 1
    return {k[n:]: v for k, v in d.items() if k.startswith(prefix + ".")}
