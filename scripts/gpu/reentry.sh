#!/bin/bash
# re-entry check after a rebuild: smoke, 1-GPU bench (8-cfg fp32 headline, 1-cfg, bf16 diag)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/re_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/re_bench8.json 2> gpurun_out/re_bench8.err || exit $?
cat gpurun_out/re_bench8.json
timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/re_bench1.json 2> gpurun_out/re_bench1.err || exit $?
cat gpurun_out/re_bench1.json
