R="build/bin/reduction --method=SUM --type=double --n=1000000000 --fill=device --iterations=10 --noverify --log=none"
tools/gpu_steps.sh \
 "pytest_gpu_all|900|python -m pytest tests -q -m gpu" \
 "pmc_sq|300|rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o run --output-format csv -- $R" \
 "pmc_tcc|300|rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_tcc -o run --output-format csv -- $R" \
 "pmc_valubusy|300|rocprofv3 --pmc VALUBusy -d gpurun_out/pmc_valu -o run --output-format csv -- $R"
