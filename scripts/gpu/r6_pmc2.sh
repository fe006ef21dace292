#!/bin/bash
# Round 6 end: SQ counters of the fp32 GEMMs on the end build (lean
# epilogues), same shapes as scripts/gpu/r6_pmc.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r6pmc2
mkdir -p "$OUT"
PMC_G=8 PMC_OUT=r6pmc2/c8 PMC_SHAPES="32,28,28,64,64,3,1,1 32,14,14,128,512,1,1,0 32,7,7,1024,256,1,1,0" \
  bash scripts/gpu/conv32_pmc2.sh || exit 1
PMC_G=1 PMC_OUT=r6pmc2/c1 PMC_SHAPES="32,7,7,1024,256,1,1,0 32,4,4,512,2048,1,1,0 32,28,28,64,64,3,1,1" \
  bash scripts/gpu/conv32_pmc2.sh || exit 1
for D in c8 c1; do
  for SH in $(ls "$OUT/$D" | grep '^a_' | sed 's/^a_//'); do
    python3 -m cerebro_ds_kpgi_amd.tools.pmc_table "$OUT/$D/a_$SH" "$OUT/$D/b_$SH" \
      > "$OUT/$D/table_$SH.md" 2>&1 || exit 1
  done
done
echo done
