"""cerebro_ds_kpgi_amd — an MI355X-native model-selection training engine.

Model Hopper Parallelism (MOP) on one node of MI355X GPUs:

* every GPU pins its data partitions in HBM (``data.store``),
* S training configurations hop between partitions every sub-epoch
  (``scheduler``), shipped as flat parameter arenas by RCCL point-to-point
  send/recv over xGMI (``parallel.hop``),
* configurations with the same architecture that sit on the same GPU are
  *packed* into one horizontally-fused model, so every kernel launch trains
  all of them at once (``models.packed``), and
* the train step runs on hand-written CDNA4 HIP kernels (``ops``), with the
  PyTorch implementation of each op kept as the numerical oracle.

Capability parity target: TrellixVulnTeam/cerebro-ds_KPGI.
"""

__version__ = "0.1.0"
