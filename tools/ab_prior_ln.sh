#!/bin/bash
# A/B of the prior train step with the LayerNorm-fused sequence-linear launches (default) and with the two-launch
# form (vqa_lib.seqlin_fused_ln_ok patched to False), same library, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PKG=vae-based-music--deep-generative-models_amd
for r in 1 2; do
  timeout -k 10 300 python tools/bench_prior.py --no-cpu --only train > gpurun_out/pb.json 2>gpurun_out/pb.err || { echo "bench failed"; exit 1; }
  echo "fused   $(python -c 'import json; d=json.loads(open("gpurun_out/pb.json").read().strip().splitlines()[0]); print(d["ms_per_step"], d["loss"])')"
  timeout -k 10 300 python -c "
import runpy, sys
sys.path.insert(0, '$PKG')
import vqa_lib
vqa_lib.seqlin_fused_ln_ok = lambda *a: False
sys.argv = ['bench_prior.py', '--no-cpu', '--only', 'train']
runpy.run_path('tools/bench_prior.py', run_name='__main__')" > gpurun_out/pb.json 2>gpurun_out/pb.err || { echo "bench failed"; exit 1; }
  echo "unfused $(python -c 'import json; d=json.loads(open("gpurun_out/pb.json").read().strip().splitlines()[0]); print(d["ms_per_step"], d["loss"])')"
done
