#!/bin/bash
# one-config packs: wgrad batch rows per split
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rows1
for R in 1 2; do
for W in 1024 512 768 1536; do
  CER_WGB_ROWS=$W timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/rows1/b1_r${W}_$R.json 2> gpurun_out/rows1/b1_r${W}_$R.err || exit $?
  echo "cfg=1 rows=$W: $(python -c "import json;d=json.load(open('gpurun_out/rows1/b1_r${W}_$R.json'));print(d['value'],d['ms_per_step'])")"
done
done
