#!/bin/bash
# Run one command against the product library and against variant libraries (copied over the in-tree libvqa.so
# in turn; the product library is restored at the end). Usage: tools/lib_ab.sh "COMMAND" VARIANT.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
CMD=$1; shift
cp $L /tmp/lib_ab_base.so
for v in /tmp/lib_ab_base.so "$@"; do
  cp "$v" $L
  echo "== $(basename $v)"
  timeout -k 10 300 bash -c "$CMD"
  rc=$?
  if [ $rc -ne 0 ]; then cp /tmp/lib_ab_base.so $L; echo "failed ($rc)"; exit $rc; fi
done
cp /tmp/lib_ab_base.so $L
