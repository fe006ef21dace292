from .base import InvariantMonitor, MOPScheduler, SchedulerInvariantError  # noqa: F401
from .policies import (GreedyScheduler, RotationScheduler, TaskParallelScheduler,  # noqa: F401
                       make_scheduler, rotate)
from .simulator import (bernoulli_runtimes, predict_greedy_runtime,  # noqa: F401
                        predict_rotation_runtime, simulate_greedy, simulate_rotation, sweep)
