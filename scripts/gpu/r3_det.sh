#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for S in 0 8; do CER_BN_ATOMIC_SLABS=$S timeout -k 10 200 python3 scripts/debug/slab_determinism.py 2>&1 | tail -1 || exit 1; done
