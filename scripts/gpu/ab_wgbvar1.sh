#!/bin/bash
# one-config packs: batched wgrad tile variant (CER_WGB_VARIANT)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wgbvar1
for R in 1 2; do
for V in 1 0 2 12 14; do
  CER_WGB_VARIANT=$V timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/wgbvar1/b1_v${V}_$R.json 2> gpurun_out/wgbvar1/b1_v${V}_$R.err || exit $?
  echo "cfg=1 variant=$V: $(python -c "import json;d=json.load(open('gpurun_out/wgbvar1/b1_v${V}_$R.json'));print(d['value'],d['ms_per_step'])")"
done
done
