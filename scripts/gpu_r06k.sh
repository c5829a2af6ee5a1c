# round-6: counters of the fused LSTM sequence kernels, 8-wave form (OUZ_LSTM_SEQ_WAVES=8) (scripts/exp/lstm_seq_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r06k; mkdir -p gpurun_out/r06k
export TMPDIR=/tmp
export OUZ_LSTM_SEQ_WAVES=8
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06k/stats -o run --output-format csv -- \
  python3 scripts/exp/lstm_seq_probe.py --iters 10 > gpurun_out/r06k/stats.log 2>&1 || exit 1
k=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT"; do
  k=$((k + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $GRAFT_REPO_ROOT/gpurun_out/r06k/p$k -o run --output-format csv -- \
    python3 scripts/exp/lstm_seq_probe.py --iters 3 > gpurun_out/r06k/p$k.log 2>&1 || { echo "pass $k failed"; tail -5 gpurun_out/r06k/p$k.log; exit 1; }
done
echo ok
