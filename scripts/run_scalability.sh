#!/bin/bash
# Scalability sweep 1/2/4/8 GPUs, 1 epoch, 8-config ResNet-50 (reference run_scalability.sh:16-151).
TS=${1:-$(date "+%Y_%m_%d_%H_%M_%S")}
for size in 1 2 4 8; do
    bash "$(dirname "$0")/run_scalability_size.sh" "$TS/$size" 1 "$size" "${2:-}"
done
