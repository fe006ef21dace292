#!/bin/bash
# rehearsal of the multi-rank path on a 1-GPU box: 2 ranks wrapped onto cuda:0
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/n2
export NCCL_DEBUG=WARN
timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/n2/nccl.json 2> gpurun_out/n2/nccl.err
rc=$?
echo "nccl rc=$rc"; tail -1 gpurun_out/n2/nccl.json; grep -i -E "error|warn|duplicate" gpurun_out/n2/nccl.err | head -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
CER_ALLOW_DEVICE_WRAP=1 CER_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/n2/gloo.json 2> gpurun_out/n2/gloo.err
rc=$?
echo "gloo rc=$rc"; tail -1 gpurun_out/n2/gloo.json; grep -i -E "error" gpurun_out/n2/gloo.err | head -8
exit $rc
