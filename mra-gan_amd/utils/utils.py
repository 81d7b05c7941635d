"""Small helpers (reference utils/utils.py:5-32)."""
import os
from collections import OrderedDict


def mkdir(path):
    if not os.path.exists(path):
        os.makedirs(path)


def mkdirs(paths):
    if isinstance(paths, (list, tuple)) and not isinstance(paths, str):
        for p in paths:
            mkdir(p)
    else:
        mkdir(paths)


def new_state_dict(state_dict):
    """Strip a DataParallel 'module.' prefix from state_dict keys."""
    out = OrderedDict()
    for k, v in state_dict.items():
        out[k[7:] if k.startswith('module.') else k] = v
    return out
