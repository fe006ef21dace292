#!/bin/bash
# DA ETL at scale on the GPU box: one FULL 160 160-image ImageNet-112
# partition as Greenplum heap / TOAST / pglz pages (float32 payload, the
# reference's packed table), read through the windowed loader into HBM;
# then an 8-partition DA-Cerebro epoch (8 configs) with ETL timed separately.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3da
R=/tmp/cer_da_full
rm -rf $R; mkdir -p $R
df -h /tmp | tail -1 > gpurun_out/r3da/df.txt
nproc >> gpurun_out/r3da/df.txt
cat gpurun_out/r3da/df.txt
( time timeout -k 10 420 python -u -m cerebro_ds_kpgi_amd.tools.make_da_data --root $R/full \
    --partitions 1 --dataset imagenet --train 160160 --valid 6250 ) > gpurun_out/r3da/make_full.log 2>&1 || { tail -5 gpurun_out/r3da/make_full.log; rm -rf $R; exit 1; }
du -sh $R/full >> gpurun_out/r3da/make_full.log
tail -5 gpurun_out/r3da/make_full.log
for T in 16 8; do
  timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root $R/full --threads $T \
    > gpurun_out/r3da/etl_full_t$T.json 2> gpurun_out/r3da/etl_full_t$T.err || { tail -5 gpurun_out/r3da/etl_full_t$T.err; rm -rf $R; exit 1; }
  cat gpurun_out/r3da/etl_full_t$T.json
done
rm -rf $R/full
if [ -n "$DA_ONLY_FULL" ]; then rm -rf $R; exit 0; fi
NT=${1:-16384}
( time timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.make_da_data --root $R/da8 \
    --partitions 8 --dataset imagenet --train $NT --valid 640 ) > gpurun_out/r3da/make8.log 2>&1 || { tail -5 gpurun_out/r3da/make8.log; rm -rf $R; exit 1; }
du -sh $R/da8 >> gpurun_out/r3da/make8.log
tail -3 gpurun_out/r3da/make8.log
echo "cerebro-da, Start time: $(date "+%Y-%m-%d %H:%M:%S")" > gpurun_out/r3da/global.log
timeout -k 10 400 python -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone --run \
  --num_epochs 1 --drill_down_scalability --size 1 --backend hip --da --da_root $R/da8 \
  --train_per_partition $NT --valid_per_partition 640 \
  --logs_root gpurun_out/r3da/cerebro-da --models_root $R/models > gpurun_out/r3da/client.log 2>&1
rc=$?
echo "cerebro-da, End time: $(date "+%Y-%m-%d %H:%M:%S")" >> gpurun_out/r3da/global.log
grep SUMMARY gpurun_out/r3da/client.log | tail -1 | cut -c1-900
rm -rf $R
exit $rc
