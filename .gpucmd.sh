cd /root/repo
timeout -k 10 300 python -m pytest tests/test_gpu_transformer.py -q -m gpu > gpurun_out/t8.log 2>&1; echo "tests rc=$?" >> gpurun_out/t8.log
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase5.json 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench6.log 2>&1
tail -3 gpurun_out/t8.log; head -9 gpurun_out/phase5.json; tail -1 gpurun_out/bench6.log
