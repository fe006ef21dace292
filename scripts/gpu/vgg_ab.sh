# VGG bias-act links / PAD8 stem and the strided-dgrad zero fill: numerics,
# then same-box A/Bs (VGG-16 8 configs: links on/off, PAD8 stem on/off)
# and a VGG-16 kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/vgg1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_vgg_links_gpu.py tests/test_fp32_gpu.py > $O/tests.log 2>&1
RC=$?
grep -E "passed|failed|Error|error|vgg16 grad|stem \(" $O/tests.log | tail -15
[ $RC -ne 0 ] && exit $RC
for L in 1 0 1 0; do
  CER_BIAS_LINKS=$L timeout -k 10 300 python -u bench.py --model vgg16 > $O/b_l$L.json 2> $O/b_l$L.err || exit $?
  echo "links=$L: $(python3 -c "import json;d=json.load(open('$O/b_l$L.json'));print(d['value'],d['ms_per_step'])")"
done
for V in "CER_STEM_PAD8=0" "CER_STEM_PAD8=1" "CER_STEM_PAD8=0" "CER_STEM_PAD8=1"; do
  env $V timeout -k 10 300 python -u bench.py --model vgg16 > $O/s.json 2> $O/s.err || exit $?
  echo "$V: $(python3 -c "import json;d=json.load(open('$O/s.json'));print(d['value'],d['ms_per_step'])")"
done
BENCH_ARGS="--model vgg16" bash scripts/gpu/prof_ab.sh vggprof2 8 CER_BIAS_LINKS=1
