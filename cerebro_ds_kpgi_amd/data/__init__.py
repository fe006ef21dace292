from .catalog import availability, make_data_catalog, partition_owner  # noqa: F401
from .store import PartitionStore, gather_batch, input_buffers  # noqa: F401
