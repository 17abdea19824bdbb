"""Helpers to read the committed golden fixtures (plain .npz, no pickles)."""
import os

import numpy as np
import torch

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    return np.load(os.path.join(GOLDEN_DIR, name), allow_pickle=False)


def params_of(d, prefix):
    """Reference state_dict entries stored under 'p/<prefix><key>' -> {key: tensor}."""
    full = "p/" + prefix
    return {k[len(full):]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith(full)}
