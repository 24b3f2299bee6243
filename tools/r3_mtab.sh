#!/bin/bash
# A/B of the backward's minimum tiles per workgroup (VQA_RES_MIN_TILES), alternating, same box
set -o pipefail
mkdir -p gpurun_out/mtab
for rep in 1 2 3; do
  for m in ${MTS:-4 2 1}; do
    VQA_RES_MIN_TILES=$m timeout -k 10 120 python bench.py --no-cpu-baseline --no-roofline --steps 30 > gpurun_out/mtab/m${m}_$rep.json 2> gpurun_out/mtab/m${m}_$rep.err || exit 1
    echo "min_tiles $m rep $rep: $(python -c "import json;print(json.load(open('gpurun_out/mtab/m${m}_$rep.json'))['ms_per_step'])")"
  done
done
