timeout -k 10 700 bash tools/pmc_bench.sh
