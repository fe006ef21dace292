cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in 0 1 0 1; do
CER_VALID_GRAPH=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "model_family and nobn" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/nobn_$V.log 2>&1; echo "valid_graph=$V rc=$? $(tail -1 gpurun_out/nobn_$V.log)"
done
