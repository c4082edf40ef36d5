timeout -k 10 300 python -u tools/host_profile.py --steps 100 > gpurun_out/host_profile.txt 2>&1
