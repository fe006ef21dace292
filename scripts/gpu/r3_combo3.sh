#!/bin/bash
# DA ETL re-measure after the loader fixes; batched-wgrad knobs at 1-2 configs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
DA_ONLY_FULL=1 bash scripts/gpu/r3_da_etl.sh || exit 1
bash scripts/gpu/ab.sh wgbknob "CER_NONE=0 CER_WGB_ROWS=2048 CER_WGB_ROWS=2048,CER_WGB_VARIANT=2" "1 2" 2
