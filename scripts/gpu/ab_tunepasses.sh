#!/bin/bash
# autotune timing passes per variant (CER_TUNE_PASSES)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tunepasses
for R in 1 2; do
for P in 2 4; do
  for C in 8 1; do
    CER_TUNE_PASSES=$P timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/tunepasses/b${C}_p${P}_$R.json 2> gpurun_out/tunepasses/b${C}_p${P}_$R.err || exit $?
    echo "cfg=$C passes=$P: $(python -c "import json;d=json.load(open('gpurun_out/tunepasses/b${C}_p${P}_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
