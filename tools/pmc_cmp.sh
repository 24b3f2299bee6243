set -o pipefail
export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
C2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
for op in fused dgrad; do
  timeout -k 10 120 rocprofv3 --pmc $C1 --output-format csv -d gpurun_out/pmc_cmp/$op/a -o a -- python tools/conv_one.py $op 32768 1 3 > /dev/null 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/pmc_cmp/$op/b -o b -- python tools/conv_one.py $op 32768 1 3 > /dev/null 2>&1 || exit 1
done
echo done
