from .catalog import *  # noqa: F401,F403
