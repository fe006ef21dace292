#!/bin/bash
# end-of-round check: GPU tier, smoke, driver-shape bench, per-GPU work at N = 1/2/4/8
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
bash scripts/gpu/gpu_tier.sh final || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/driver.json 2> gpurun_out/final/driver.err || exit $?
cat gpurun_out/final/driver.json
for C in 8 4 2 1; do
  timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/final/c$C.json 2> gpurun_out/final/c$C.err || exit $?
  echo "configs=$C: $(python -c "import json;d=json.load(open('gpurun_out/final/c$C.json'));print(d['value'],d['ms_per_step'])")"
done
