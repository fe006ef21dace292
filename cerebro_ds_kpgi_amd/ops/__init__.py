from .backend import get_backend, set_backend, use_hip  # noqa: F401
