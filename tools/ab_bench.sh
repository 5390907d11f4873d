# A/B the step time of the in-tree library against ab/libsat_base.so (alternating, 2 rounds)
for i in 1 2; do
  for lib in "" "$PWD/ab/libsat_base.so"; do
    SAT_LIB_OVERRIDE=$lib timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('${lib:-new}'.split('/')[-1], d['ms_per_step'], d.get('loss_last'))" || exit 1
  done
done
