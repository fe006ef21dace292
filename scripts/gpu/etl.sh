#!/bin/bash
# Direct-Access ETL on the GPU box: write Greenplum-format heap/TOAST pages
# for 8 ImageNet-112 partitions (float32 payload, the reference's packed
# table), then one DA-Cerebro epoch (8 configs) reading them through the C++
# page / TOAST / pglz reader into HBM; the run summary carries decode / H2D
# GB/s.  Also the Criteo (16-config confA) grid through DA on the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/etl
R=/tmp/cer_etl
rm -rf $R; mkdir -p $R
NT=${1:-4096}
( time timeout -k 10 600 python -u -m cerebro_ds_kpgi_amd.tools.make_da_data --root $R/da \
    --partitions 8 --dataset imagenet --train $NT --valid 256 ) > gpurun_out/etl/make.log 2>&1 || exit $?
du -sh $R/da >> gpurun_out/etl/make.log
tail -5 gpurun_out/etl/make.log
timeout -k 10 600 python -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone --run \
  --num_epochs 1 --drill_down_scalability --size 1 --backend hip --da --da_root $R/da \
  --train_per_partition $NT --valid_per_partition 256 \
  --logs_root gpurun_out/etl/cerebro-da --models_root $R/models > gpurun_out/etl/client.log 2>&1 || exit $?
grep SUMMARY gpurun_out/etl/client.log | tail -1
rm -rf $R
timeout -k 10 600 python -u bench.py --workload criteo16 --da > gpurun_out/etl/bench_criteo_da.json \
  2> gpurun_out/etl/bench_criteo_da.err || exit $?
cat gpurun_out/etl/bench_criteo_da.json
