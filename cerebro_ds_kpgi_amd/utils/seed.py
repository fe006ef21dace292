"""Process-wide seeding (reference ``cerebro_gpdb/utils.py:152-201``).

The reference's ``set_seed`` has a latent NameError on its TF fallback path
(``seed_value``); this one seeds python, numpy and torch unconditionally.
"""

import os
import random

import numpy as np

from ..config.catalog import SEED


def set_seed(seed=SEED, backend="pytorch"):
    os.environ["PYTHONHASHSEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed)
    try:
        import torch
        torch.manual_seed(seed)
    except ImportError:  # pragma: no cover
        pass
    return seed
