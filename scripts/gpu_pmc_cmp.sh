# MMQ prefill counters, f16 tile vs int8 tile (one --pmc pass per group)
export PMCS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS|TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE|TCC_EA0_RDREQ_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum|SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
export KRE=k_mmq_q4K
bash scripts/gpu_pmc_mmq.sh > gpurun_out/pmc_f16.txt 2>&1 || { cat gpurun_out/pmc_f16.txt; exit 1; }
GGML_MI355X_MMQ_F16=0 bash scripts/gpu_pmc_mmq.sh > gpurun_out/pmc_i8.txt 2>&1 || { cat gpurun_out/pmc_i8.txt; exit 1; }
cat gpurun_out/pmc_f16.txt gpurun_out/pmc_i8.txt
