#!/bin/bash
# r04 GPU call F: kernel stats of the launch-bound Flickr config and of products k = 32 with the
# edge-selector stream (now on by default there), and the products k = 32 / 64 presets refreshed
# with their denominators.
set -eo pipefail
cd "$(dirname "$0")/.."
CFGS="flickr:--graph flickr products_k32:--graph products --k 32" bash tools/session.sh r04 statscfg
mkdir -p gpurun_out/r04/presets
O=gpurun_out/r04
for k in 32 64; do
  timeout -k 10 400 python bench.py --cpu-seconds 6 --graph products --k $k \
    > $O/presets/products_k$k.json 2> $O/presets/products_k$k.err
  echo "products k=$k: $(cut -c1-200 $O/presets/products_k$k.json)"
done
