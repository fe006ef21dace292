#!/bin/bash
# probe: does running config packs concurrently (separate processes -> separate HW queues)
# beat one 8-config pack?  Sum of concurrent img/s vs single.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/conc
timeout -k 10 300 python -u bench.py --steps 100 > gpurun_out/conc/c8.json 2> gpurun_out/conc/c8.err || exit $?
echo "single 8cfg: $(python -c "import json;print(json.load(open('gpurun_out/conc/c8.json'))['value'])")"
timeout -k 10 300 python -u bench.py --configs 4 --steps 100 > gpurun_out/conc/c4.json 2> gpurun_out/conc/c4.err || exit $?
echo "single 4cfg: $(python -c "import json;print(json.load(open('gpurun_out/conc/c4.json'))['value'])")"
pids=""
for i in 0 1; do
  timeout -k 10 300 python -u bench.py --configs 4 --steps 200 --warmup 40 > gpurun_out/conc/p4_$i.json 2> gpurun_out/conc/p4_$i.err &
  pids="$pids $!"
done
rc=0; for p in $pids; do wait $p || rc=$?; done
[ $rc -ne 0 ] && exit $rc
echo "2 x 4cfg concurrent: $(python -c "import json;print([json.load(open('gpurun_out/conc/p4_%d.json'%i))['value'] for i in (0,1)])")"
pids=""
for i in 0 1 2 3; do
  timeout -k 10 300 python -u bench.py --configs 2 --steps 300 --warmup 60 > gpurun_out/conc/p2_$i.json 2> gpurun_out/conc/p2_$i.err &
  pids="$pids $!"
done
rc=0; for p in $pids; do wait $p || rc=$?; done
[ $rc -ne 0 ] && exit $rc
echo "4 x 2cfg concurrent: $(python -c "import json;print([json.load(open('gpurun_out/conc/p2_%d.json'%i))['value'] for i in range(4)])")"
