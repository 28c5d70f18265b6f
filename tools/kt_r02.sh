#!/bin/bash
# The reference's kernel-test comparison (maxk_kernel_test.py) on every config graph.
set -eo pipefail
mkdir -p gpurun_out/kt
for g in reddit products proteins; do
  timeout -k 10 300 python spgemm-prunning_amd/maxk_kernel_test.py $g --k 8 16 32 64 --json > gpurun_out/kt/$g.txt 2> gpurun_out/kt/$g.err
done
timeout -k 10 300 python spgemm-prunning_amd/maxk_kernel_test.py flickr --dim 64 --k 8 16 32 64 --json > gpurun_out/kt/flickr.txt 2> gpurun_out/kt/flickr.err
echo kt done
