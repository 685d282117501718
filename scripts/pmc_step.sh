#!/bin/bash
# PMC wait/issue breakdown of every kernel of one eager Base step
# (scripts/layer_profile.py), three counter passes; summary per kernel
# template instance: gpurun_out/pmc_step_summary.txt
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="python3 scripts/layer_profile.py --top 1"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmcs_c$i -o run -- $C > gpurun_out/pmcs_c$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmcs_c$i.log; exit 1; }
done
for f in wgrad3x3_halo conv3x3_hs conv3x3_ws stem_ maxpool bn_ head_; do
  python3 scripts/pmc_summary.py $f gpurun_out/pmcs_c1 gpurun_out/pmcs_c2 gpurun_out/pmcs_c3
done > gpurun_out/pmc_step_summary.txt 2>&1
rm -rf gpurun_out/pmcs_c*/
