cd /root/repo
timeout -k 10 300 python -m pytest tests/test_gpu_transformer.py -q -m gpu > gpurun_out/t4.log 2>&1; echo "tests rc=$?" >> gpurun_out/t4.log
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > gpurun_out/bench2.log 2>&1; echo "bench rc=$?" >> gpurun_out/bench2.log
tail -3 gpurun_out/t4.log; tail -2 gpurun_out/bench2.log
