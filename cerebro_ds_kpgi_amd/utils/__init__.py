from .logging import LOG_KEYS, DiskLogs, GlobalLog, logs, logsc, timeit_factory, tstamp  # noqa: F401
from .keys import key2mst, model_key, mst2key, mst_2_str  # noqa: F401
from .seed import set_seed  # noqa: F401
