# SQ/TCC counters of one kernel family (KRE) during a pp512 bench (one --pmc pass per group)
export PMCS="${PMCS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS|SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU|TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE}"
bash scripts/gpu_pmc_mmq.sh > gpurun_out/pmc_one.txt 2>&1 || { cat gpurun_out/pmc_one.txt; exit 1; }
cat gpurun_out/pmc_one.txt
