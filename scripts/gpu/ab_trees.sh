#!/bin/bash
# Same-lease A/B of two whole builds (Python + native libraries), e.g. the
# round-4 end tree against HEAD:
#
#   bash scripts/gpu/ab_trees.sh NAME "TREE_A TREE_B" [ROUNDS] ["WORKLOADS"]
#
# Each TREE is a directory holding a built checkout (abtree/r4 = `git archive
# 75bda2a` built in place with its own tools.build; "." = this tree).  Every
# round runs each workload on each tree, alternating, with the driver's bench
# shape (`--gpus 1 --steps 20 --warmup 5`); workload "c1" = the headline with
# --configs 1 (the N = 8 per-GPU work).  Output: gpurun_out/abt_NAME/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
NAME=${1:?name}
TREES=${2:?trees}
ROUNDS=${3:-3}
WORKLOADS=${4:-"headline criteo16"}
OUT=$PWD/gpurun_out/abt_$NAME
mkdir -p "$OUT"
for R in $(seq 1 "$ROUNDS"); do
  for W in $WORKLOADS; do
    for T in $TREES; do
      TAG=${T//[\/.]/_}
      F="$OUT/b_${TAG}_${W}_$R"
      case $W in
        c1) ARGS="--workload headline --configs 1" ;;   # the N = 8 per-GPU work
        *) ARGS="--workload $W" ;;
      esac
      (cd "$T" && timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
         $ARGS > "$F.json" 2> "$F.err") || { tail -20 "$F.err"; exit 1; }
      echo "$T $W r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
