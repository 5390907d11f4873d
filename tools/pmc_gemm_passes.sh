# PMC passes (MFMA pipe busy, wave states, LDS conflicts) of the LDS GEMM kernel on the step's
# largest product shapes, planner-chosen plans; run on the GPU box from the repo root:
#   bash tools/pmc_gemm_passes.sh   ->  gpurun_out/pmc_lds/summary.jsonl
set -e
OUT=gpurun_out/pmc_lds
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
for shape in "16000 1024 256 0" "16000 256 1024 0" "544 1024 16000 1" "16000 1024 544 0"; do
  set -- $shape
  tag=s$1_$2_$3_$4
  timeout -s KILL 60 rocprofv3 --pmc $P1 --kernel-trace -d $OUT/${tag}_p1 -o pmc -- python3 tools/pmc_gemm.py run $1 $2 $3 $4 > /dev/null 2>&1
  timeout -s KILL 60 rocprofv3 --pmc $P2 --kernel-trace -d $OUT/${tag}_p2 -o pmc -- python3 tools/pmc_gemm.py run $1 $2 $3 $4 > /dev/null 2>&1
  python3 tools/pmc_gemm.py summary $OUT $tag $1 $2 $3 >> $OUT/summary.jsonl
done
cat $OUT/summary.jsonl
