#!/bin/bash
# round 3 first probe: graph launch floor, 1-config timeline profile, c1/c8 bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3probe
timeout -k 10 200 python -u -m cerebro_ds_kpgi_amd.tools.launch_floor > gpurun_out/r3probe/floor.json 2> gpurun_out/r3probe/floor.err || exit $?
cat gpurun_out/r3probe/floor.json
for C in 1 8; do
  timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/r3probe/c$C.json 2> gpurun_out/r3probe/c$C.err || exit $?
  echo "c$C $(python3 -c "import json;d=json.load(open('gpurun_out/r3probe/c$C.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3probe/prof_c1 -o prof -- \
  python3 bench.py --steps 20 --warmup 10 --steps_per_round 10 --configs 1 > gpurun_out/r3probe/prof_c1.log 2>&1 || exit $?
tail -1 gpurun_out/r3probe/prof_c1.log
