#!/bin/bash
# Round 4 first call: can RCCL run several ranks on one GPU (a real-RCCL
# rehearsal of the hop data plane), plus the driver-shape bench on the
# round-3 build as this round's starting point.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/probe
mkdir -p $out
for n in 2 4; do
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) scripts/dev/rccl_probe.py \
    > $out/rccl_probe_n$n.log 2>&1
  echo "rccl probe n=$n exit $?" | tee -a $out/summary.txt
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
echo "bench exit $?" | tee -a $out/summary.txt
cat $out/bench.json
