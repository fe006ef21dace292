# VGG bias-act links / PAD8 stem and the strided-dgrad zero fill: numerics,
# then same-box A/Bs (VGG-16 8 configs links on/off; ResNet-50 zfill on/off)
# and a VGG-16 kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/vgg1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_vgg_links_gpu.py tests/test_zfill_gpu.py tests/test_fp32_gpu.py > $O/tests.log 2>&1
RC=$?
grep -E "passed|failed|Error|error|vgg16 grad|stem \(" $O/tests.log | tail -15
[ $RC -ne 0 ] && exit $RC
for L in 1 0 1 0; do
  CER_BIAS_LINKS=$L timeout -k 10 300 python -u bench.py --model vgg16 > $O/b_l$L.json 2> $O/b_l$L.err || exit $?
  echo "links=$L: $(python3 -c "import json;d=json.load(open('$O/b_l$L.json'));print(d['value'],d['ms_per_step'])")"
done
for Z in 1 0 1 0; do
  for C in 1 8; do
    CER_DGRAD_ZFILL=$Z timeout -k 10 300 python -u bench.py --configs $C > $O/r_z${Z}_c$C.json 2> $O/r_z${Z}_c$C.err || exit $?
    echo "zfill=$Z configs=$C: $(python3 -c "import json;d=json.load(open('$O/r_z${Z}_c$C.json'));print(d['value'],d['ms_per_step'])")"
  done
done
BENCH_ARGS="--model vgg16" bash scripts/gpu/prof_ab.sh vggprof2 8 CER_BIAS_LINKS=1
