# Round evidence on one MI355X (run on the GPU box from the repo root):
#   bash tools/round_evidence.sh TAG
# -> gpurun_out/TAG_{gputest.log,smoke.log,bench.json,prof/,timeline.txt,stats_top.txt}
#    and the PMC summaries (pmc_attn/summary.json, pmc_lds/summary.jsonl).
# Each GPU step has its own time limit; a fault / abort / time-out ends the script there.
TAG=${1:-r04}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
stop() {  # exit codes of a GPU fault, abort, segfault or time-out end the call
  case $1 in 124|134|137|139) echo "step '$2' ended with $1: stopping"; exit $1;; esac
}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > $O/${TAG}_gputest.log 2>&1; rc=$?; tail -3 $O/${TAG}_gputest.log; stop $rc gputest
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
rc=$?; tail -2 $O/${TAG}_smoke.log; stop $rc smoke
timeout -k 10 400 python -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err; rc=$?
tail -c 600 $O/${TAG}_bench.json; stop $rc bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra \
  > $O/${TAG}_prof_bench.json 2> $O/${TAG}_prof.err; rc=$?; stop $rc rocprof
python3 tools/step_timeline.py $O/${TAG}_prof/run_kernel_trace.csv --list > $O/${TAG}_timeline.txt 2>&1
python3 tools/stats_top.py $O/${TAG}_prof/run_kernel_stats.csv \
  "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra" 40 \
  > $O/${TAG}_stats_top.txt 2>&1
head -4 $O/${TAG}_timeline.txt
bash tools/pmc_attn_fwd.sh > /dev/null 2>&1; rc=$?; stop $rc pmc_attn
cat $O/pmc_attn/summary.json 2>/dev/null | head -c 400; echo
bash tools/pmc_gemm_passes.sh > /dev/null 2>&1; rc=$?; stop $rc pmc_gemm
cat $O/pmc_lds/summary.jsonl 2>/dev/null | cut -c1-300
echo done
