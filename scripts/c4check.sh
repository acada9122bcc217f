# class-loop change check: affinity parity, full-size digests (C1-C4), C4 bench
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py tests/test_affinity_errors.py -k "affinity or golden or c4 or error" > gpurun_out/aff_tests.log 2>&1; rc=$?; tail -3 gpurun_out/aff_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -m gpu -v -p no:cacheprovider -x --timeout 300 --timeout-method thread tests/test_gpu_digest.py > gpurun_out/digest_tests.log 2>&1; rc=$?; tail -8 gpurun_out/digest_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-eval > gpurun_out/bench_C4.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_C4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_us_per_launch'])"
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval > gpurun_out/bench_C4_diag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_C4_diag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('diag_place_phases'), d['roofline']['avg_us_per_launch'], d['value'])"
