# PMC passes of the LDS GEMM kernel at forced plans (run on the GPU box from the repo root).
set -e
mkdir -p gpurun_out/pmc2
P1="SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
for plan in 128,128,1 64,64,1; do
  tag=p$(echo $plan | tr , _)
  SAT_GEMM_PLAN=$plan timeout -s KILL 60 rocprofv3 --pmc $P1 --kernel-trace -d gpurun_out/pmc2/${tag}_p1 -o pmc -- python3 tools/pmc_gemm.py run 16000 1024 256 > /dev/null 2>&1
  SAT_GEMM_PLAN=$plan timeout -s KILL 60 rocprofv3 --pmc $P2 --kernel-trace -d gpurun_out/pmc2/${tag}_p2 -o pmc -- python3 tools/pmc_gemm.py run 16000 1024 256 > /dev/null 2>&1
  python3 tools/pmc_gemm.py summary gpurun_out/pmc2 $tag 16000 1024 256 >> gpurun_out/pmc2/summary.jsonl
done
cat gpurun_out/pmc2/summary.jsonl
