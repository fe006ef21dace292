#!/bin/bash
# bf16 graph-replay test with / without the shortcut branch stream, then the
# full tier and the bit-mask A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s7
for B in 0 1 1; do
  CER_SC_BRANCH=$B timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -q --timeout 200 \
    --timeout-method thread -k "fwd_bwd_graph_replays_equal_eager" > gpurun_out/r3s7/graph_b$B.log 2>&1
  echo "branch=$B: $(tail -1 gpurun_out/r3s7/graph_b$B.log)"
  grep -E "^E  .*assert" gpurun_out/r3s7/graph_b$B.log | head -3
done
bash scripts/gpu/gpu_tier.sh r3s7
bash scripts/gpu/ab.sh bitmask "CER_BN_BITMASK=0 CER_BN_BITMASK=1" "1 8" 2
