cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
b() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])' 2>/dev/null)"; return $rc; }
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 b p25nopkt python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipeline-chunk 25 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 b seqnopkt python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipeline-chunk 0 &&
b seq_eager python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipeline-chunk 0 --no-graph &&
b p25_eager python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipeline-chunk 25 --no-graph
