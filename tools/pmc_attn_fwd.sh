# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the persistent attention forward in
# the bench configuration; run on the GPU box from the repo root:
#   bash tools/pmc_attn_fwd.sh  ->  gpurun_out/pmc_attn/summary.json
set -e
OUT=gpurun_out/pmc_attn
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o pmc -- python3 tools/pmc_persistent.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o pmc -- python3 tools/pmc_persistent.py > /dev/null 2>&1
python3 tools/pmc_summary.py $OUT/fetch $OUT/write dec_attn_fwd8_kernel > $OUT/summary.json
cat $OUT/summary.json
