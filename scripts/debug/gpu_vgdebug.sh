cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for M in resnet50_nobn resnet18 vgg16; do
  for E in "CER_VALID_GRAPH=1" "CER_VALID_GRAPH=1 CER_WGRAD_BATCH=0" "CER_VALID_GRAPH=1 CER_CONV_TUNE=0"; do
    env $E timeout -k 10 200 python scripts/debug/valid_graph_nan.py $M > gpurun_out/vg_$M.log 2>&1 || { echo "fail $M $E"; tail -5 gpurun_out/vg_$M.log; exit 1; }
    echo "$M [$E]: $(grep 'epoch 1 model 0' gpurun_out/vg_$M.log)"
  done
done
