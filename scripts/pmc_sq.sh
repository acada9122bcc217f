set -u
export TMPDIR=/tmp
OUT=gpurun_out
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-timing --path select"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $PWD/$OUT/pmc1 -o run --output-format csv -- $B > $OUT/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_MISSES -d $PWD/$OUT/pmc2 -o run --output-format csv -- $B > $OUT/pmc2.log 2>&1 || exit 1
echo ok
