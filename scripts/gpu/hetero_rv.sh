#!/bin/bash
# BASELINE config 4: the heterogeneous {ResNet-50, VGG-16} x {lr, batch 32 / 64}
# 8-config grid (param_grid_hetero_rv) as real jobs at N = 1 -- greedy (CTQ,
# runners.ctq) and rotation (UDAF, runners.run_mop) on 8 reduced partitions --
# plus the per-class pack step times (bench.py, 1 and 2 configs) that
# tools.hetero_project turns into the N = 2 / 4 / 8 greedy-vs-rotation table.
#   bash scripts/gpu/hetero_rv.sh [TRAIN_PER_PARTITION]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/hetero_rv
TP=${1:-2048}
mkdir -p $O
CLS=""
for MB in resnet50:32 resnet50:64 vgg16:32 vgg16:64; do
  M=${MB%%:*}; B=${MB##*:}
  for C in 1 2; do
    timeout -k 10 400 python3 -u bench.py --model $M --batch $B --configs $C --steps 20 --warmup 5 \
      --steps_per_round 10 > $O/rate_${M}_b${B}_c$C.json 2> $O/rate_${M}_b${B}_c$C.err || { tail -5 $O/rate_${M}_b${B}_c$C.err; exit 1; }
  done
  T1=$(python3 -c "import json;print(json.load(open('$O/rate_${M}_b${B}_c1.json'))['ms_per_step']/1000)")
  T2=$(python3 -c "import json;print(json.load(open('$O/rate_${M}_b${B}_c2.json'))['ms_per_step']/1000)")
  echo "$M bs$B: step ${T1}s (1 config) ${T2}s (2 configs)"
  CLS="$CLS;${M}_b$B,2,$B,$T1,$T2,2"
done
for A in ctq run_mop; do
  timeout -k 10 900 python3 -u -m cerebro_ds_kpgi_amd.runners.$A --run --num_epochs 1 \
    --drill_down_hetero_rv --size 1 --slots_per_gpu 8 --train_per_partition $TP \
    --valid_per_partition $((TP / 25)) --backend hip --logs_root $O/$A/logs \
    --models_root /tmp/hrv_models > $O/$A.log 2>&1 || { tail -20 $O/$A.log; exit 1; }
  grep SUMMARY $O/$A.log | tail -1 | cut -c1-400
  rm -rf /tmp/hrv_models
done
python3 -m cerebro_ds_kpgi_amd.tools.hetero_project --classes "${CLS#;}" --train_images $((8 * TP)) \
  > $O/projection.md && cat $O/projection.md
# full-size projection (one ImageNet epoch)
python3 -m cerebro_ds_kpgi_amd.tools.hetero_project --classes "${CLS#;}" > $O/projection_full.md && head -7 $O/projection_full.md
