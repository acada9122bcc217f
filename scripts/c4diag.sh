cd $GRAFT_REPO_ROOT
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval > gpurun_out/bench_C4_diag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_C4_diag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('diag_place_phases'), d['roofline']['avg_us_per_launch'], d['value'])"
