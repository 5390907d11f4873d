# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the persistent attention forward and
# BPTT in the bench configuration; run on the GPU box from the repo root:
#   bash tools/pmc_attn_fwd.sh  ->  gpurun_out/pmc_attn/{summary,summary_bwd}.json
set -e
OUT=gpurun_out/pmc_attn
C=self-attention-tacotron_amd/csrc
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o pmc -- python3 tools/pmc_persistent.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o pmc -- python3 tools/pmc_persistent.py > /dev/null 2>&1
python3 tools/pmc_summary.py $OUT/fetch $OUT/write dec_attn_fwd8_kernel $C/decoder_persistent8.hip > $OUT/summary.json
python3 tools/pmc_summary.py $OUT/fetch $OUT/write dec_attn_bwd8_kernel $C/decoder_persistent8_bwd.hip > $OUT/summary_bwd.json
cat $OUT/summary.json $OUT/summary_bwd.json
