#!/bin/bash
# the driver's bench shape on a fresh box, then the secondary BASELINE workloads (fp32)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/bench_all
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_all/driver_shape.json 2> gpurun_out/bench_all/driver_shape.err || exit $?
cat gpurun_out/bench_all/driver_shape.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_all/default.json 2> gpurun_out/bench_all/default.err || exit $?
cat gpurun_out/bench_all/default.json
for W in hetero8 criteo16; do
  timeout -k 10 400 python3 bench.py --workload $W > gpurun_out/bench_all/$W.json 2> gpurun_out/bench_all/$W.err || exit $?
  cat gpurun_out/bench_all/$W.json
done
