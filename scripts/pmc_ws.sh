# PMC breakdown of the weight-stationary halo conv on enc1 (fwd + dgrad) and dec1.3
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="python3 scripts/tune_conv.py --reps 2 --cfgs 0 --only enc1_3x3,dec1.3 --modes 0,1 --epi"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
           "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmcws_c$i -o run -- $C > gpurun_out/pmcws_c$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmcws_c$i.log; exit 1; }
done
python3 scripts/pmc_summary.py conv3x3_ws gpurun_out/pmcws_c1 gpurun_out/pmcws_c2 gpurun_out/pmcws_c3 > gpurun_out/pmcws_summary.txt
