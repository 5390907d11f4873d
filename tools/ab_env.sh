# A/B of two environment settings of the training step (alternating, 3 rounds), run from the repo
# root on the GPU box:  ENVA="X=1" ENVB="X=0" bash tools/ab_env.sh
run() { env $2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 $2', d['ms_per_step'], d.get('loss_last'))"; }
for i in 1 2 3; do run A "$ENVA" || exit 1; run B "$ENVB" || exit 1; done
