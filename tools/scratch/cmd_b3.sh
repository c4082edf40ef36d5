set -e -o pipefail
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/b3_$i.log 2>&1; done
