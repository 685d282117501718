export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="python3 scripts/tune_conv.py --reps 2 --cfgs 0 --only enc3_3x3,dec1.0 --modes 0"
i=0
for set in "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" "FETCH_SIZE WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc_c$i -o run -- $C > gpurun_out/pmc_c$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_c$i.log; exit 1; }
done
