# PMC wait/issue breakdown of the implicit-GEMM conv on enc3 fwd, tile cfgs 15 (NS=2) and 16 (NS=3)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="python3 scripts/tune_conv.py --reps 2 --cfgs 15,16 --only enc3_3x3 --modes 0 --epi"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc2_c$i -o run -- $C > gpurun_out/pmc2_c$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc2_c$i.log; exit 1; }
done
python3 scripts/pmc_summary.py conv_glds gpurun_out/pmc2_c1 gpurun_out/pmc2_c2 gpurun_out/pmc2_c3 > gpurun_out/pmc2_summary.txt
