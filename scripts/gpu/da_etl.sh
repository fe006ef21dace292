#!/bin/bash
# DA ETL at scale on the GPU box (profiles/r4_da_etl.md):
#  1. one FULL 160 160-image ImageNet-112 partition as Greenplum heap / TOAST /
#     pglz pages (float32 payload, the reference's packed table): the windowed
#     loader into HBM at 16 threads, and the C++ reader alone (decode only),
#     with the reader's per-phase timings;
#  2. the N = 8 host shape: 8 partitions read by 8 concurrent reader
#     processes (one per simulated rank, 2 threads each on this box's 16-CPU
#     share) against one reader at 16 threads over the same 8 partitions;
#  3. (arg "epoch") an 8-partition DA-Cerebro epoch with ETL timed separately.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4da
mkdir -p $O
R=/tmp/cer_da_full
rm -rf $R; mkdir -p $R
{ df -h /tmp | tail -1; nproc; free -g | head -2; } > $O/host.txt
cat $O/host.txt
( time timeout -k 10 420 python -u -m cerebro_ds_kpgi_amd.tools.make_da_data --root $R/full \
    --partitions 1 --dataset imagenet --train 160160 --valid 6250 ) > $O/make_full.log 2>&1 || { tail -5 $O/make_full.log; rm -rf $R; exit 1; }
du -sh $R/full >> $O/make_full.log
tail -4 $O/make_full.log
timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root $R/full --threads 16 \
  > $O/etl_full_t16.json 2> $O/etl_full_t16.err || { tail -5 $O/etl_full_t16.err; rm -rf $R; exit 1; }
cat $O/etl_full_t16.json
timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root $R/full --threads 16 \
  --decode_only > $O/decode_full_t16.json 2> $O/decode_full_t16.err || { tail -5 $O/decode_full_t16.err; rm -rf $R; exit 1; }
cat $O/decode_full_t16.json
rm -rf $R/full
( time timeout -k 10 420 python -u -m cerebro_ds_kpgi_amd.tools.make_da_data --root $R/da8 \
    --partitions 8 --dataset imagenet --train 32100 --valid 642 ) > $O/make8.log 2>&1 || { tail -5 $O/make8.log; rm -rf $R; exit 1; }
du -sh $R/da8 >> $O/make8.log
tail -3 $O/make8.log
timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root $R/da8 --threads 2 \
  --decode_only --concurrent 8 > $O/decode8_concurrent.json 2> $O/decode8_concurrent.err || { tail -5 $O/decode8_concurrent.err; rm -rf $R; exit 1; }
cat $O/decode8_concurrent.json
timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root $R/da8 --threads 16 \
  --decode_only > $O/decode8_t16.json 2> $O/decode8_t16.err || { tail -5 $O/decode8_t16.err; rm -rf $R; exit 1; }
cat $O/decode8_t16.json
if [ "$1" != "epoch" ]; then rm -rf $R; exit 0; fi
echo "cerebro-da, Start time: $(date "+%Y-%m-%d %H:%M:%S")" > $O/global.log
timeout -k 10 400 python -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone --run \
  --num_epochs 1 --drill_down_scalability --size 1 --backend hip --da --da_root $R/da8 \
  --train_per_partition 32100 --valid_per_partition 642 \
  --logs_root $O/cerebro-da --models_root $R/models > $O/client.log 2>&1
rc=$?
echo "cerebro-da, End time: $(date "+%Y-%m-%d %H:%M:%S")" >> $O/global.log
grep SUMMARY $O/client.log | tail -1 | cut -c1-900
rm -rf $R
exit $rc
