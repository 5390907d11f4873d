cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-600; return $rc; }
step pmcf 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python3 tools/pmc_attention.py &&
step pmcw 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o pmc -- python3 tools/pmc_attention.py &&
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_attn.json; cat gpurun_out/pmc_attn.json
