set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for arm in ${ARMS:-v7 v8 blas}; do
  timeout -s KILL 90 rocprofv3 --pmc $CTRS -d gpurun_out/pmc1_$arm -o $arm -- python3 tools/gemm_arm.py $arm 8192 20 > gpurun_out/pmc1_$arm.log 2>&1 || { echo "pmc $arm failed rc=$?"; tail -5 gpurun_out/pmc1_$arm.log; exit 1; }
done
CTRS2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for arm in ${ARMS:-v7 v8 blas}; do
  timeout -s KILL 90 rocprofv3 --pmc $CTRS2 -d gpurun_out/pmc2_$arm -o $arm -- python3 tools/gemm_arm.py $arm 8192 20 > gpurun_out/pmc2_$arm.log 2>&1 || { echo "pmc2 $arm failed rc=$?"; tail -5 gpurun_out/pmc2_$arm.log; exit 1; }
done
for p in pmc1 pmc2; do for arm in ${ARMS:-v7 v8 blas}; do
  db=$(find gpurun_out/${p}_$arm -name "*.db" | head -1)
  pat=gemm_bf16_tn; [ $arm = blas ] && pat=Cijk
  echo "=== $p $arm ($db)"; python3 tools/pmc_summary.py "$db" $pat
done; done
