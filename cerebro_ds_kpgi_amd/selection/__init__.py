from .grid import get_exp_specific_msts, get_msts  # noqa: F401
