#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/debug/grad_sens.py resnet50 4 > gpurun_out/grad_sens4.log 2>&1; echo rc=$?
cat gpurun_out/grad_sens4.log | grep -v amdgpu.ids
timeout -k 10 300 python scripts/debug/grad_sens.py resnet50 32 > gpurun_out/grad_sens32.log 2>&1; echo rc=$?
cat gpurun_out/grad_sens32.log | grep -v amdgpu.ids
