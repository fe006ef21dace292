#!/bin/bash
# GPU tier after the round-3 pruning + driver-shape bench + 1-config bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3tier
bash scripts/gpu/gpu_tier.sh ${1:-r3a} || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3tier/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3tier/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3tier/driver.json 2> gpurun_out/r3tier/driver.err || exit $?
cat gpurun_out/r3tier/driver.json
timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/r3tier/c1.json 2> gpurun_out/r3tier/c1.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r3tier/c1.json'));print('c1',d['value'],d['ms_per_step'])"
