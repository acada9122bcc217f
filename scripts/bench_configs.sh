cd $GRAFT_REPO_ROOT
for c in C1 C3 C4; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 > gpurun_out/bench_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
done
