#!/bin/bash
# Round 6 end: secondary workloads on the end build (fp32, N = 1)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6sec
mkdir -p $O
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['metric'],d['value'],d['ms_per_step'])")"
}
run criteo16 --workload criteo16
run hetero8 --workload hetero8
run e2e16 --workload e2e16 --steps 20 --warmup 5 --steps_per_round 10
for M in mobilenetv2 resnet152 vgg16; do run size_$M --model $M --steps 30 --warmup 10; done
