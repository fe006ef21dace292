from .dist import DistContext, init_distributed, shutdown  # noqa: F401
from .hop import Move, execute_moves, plan_moves, validate_plan  # noqa: F401
