#!/bin/bash
# Round-4 residual-block epilogue adds as single v_add_f32 (no packed adds beside MFMAs): resblock tests on the new
# library, forward kernel stats of both, step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r4add4
mkdir -p $OUT
L=vae-based-music--deep-generative-models_amd/libvqa.so
cp $L $OUT/base.so
cp variants/rb_add4.so $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resblock.py > $OUT/tests.log 2>&1 || { cp $OUT/base.so $L; echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
cp $OUT/base.so $L
{ tools/kt_fwd.sh $OUT/base.so base $OUT && tools/kt_fwd.sh variants/rb_add4.so add4 $OUT; } > $OUT/kt.log 2>&1 || exit 1
tools/ab_libs.sh 3 variants/rb_add4.so > $OUT/step_ab.log 2>&1
