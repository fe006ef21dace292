#!/bin/bash
# Round 6: the headline is 1.5 % below the round-4 end build in one lease
# (gpurun_out/abt_r4r6).  Same lease: round-4 tree vs this tree with the
# round-5 features that the bisect pointed at switched off by their knobs.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6regr
mkdir -p $O
for R in 1 2 3; do
  (cd abtree/r4 && timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r4_$R.json 2> $O/r4_$R.err) || exit 1
  echo "r4 r$R $(python3 -c "import json;d=json.load(open('$O/r4_$R.json'));print(d['value'],d['ms_per_step'])")"
  for V in CER_NONE=0 CER_WGB_NARROW=0 CER_DRES_LAZY=0 CER_WGB_NARROW=0,CER_DRES_LAZY=0 CER_UK=0; do
    F=$O/${V//[,=]/_}_$R
    env ${V//,/ } timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $F.json 2> $F.err || exit 1
    echo "$V r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
  done
done
