#!/bin/bash
# PMC breakdown of the halo-streamed conv (enc3 / enc4 fwd + dgrad)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="python3 scripts/tune_conv.py --reps 2 --cfgs 0 --only ${SHAPES:-enc3_3x3,enc4_3x3} --modes 0,1 --epi"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmchs_c$i -o run -- $C > gpurun_out/pmchs_c$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmchs_c$i.log; exit 1; }
done
python3 scripts/pmc_summary.py ${FILTER:-conv3x3_hs} gpurun_out/pmchs_c1 gpurun_out/pmchs_c2 gpurun_out/pmchs_c3 > gpurun_out/pmchs_summary.txt
