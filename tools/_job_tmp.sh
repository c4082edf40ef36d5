set -o pipefail
bash tools/gpu_job.sh tests "transformer or chunked or cnn or CNN or step_tables or rnn" tests/test_gpu_transformer.py tests/test_gpu_chunked.py tests/test_gpu_programs.py tests/test_gpu_rnn.py
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
rm -f gpurun_out/ph_new.txt
for wv in 0 4; do timeout -k 10 120 python tools/phase_profile.py --block 1 --wave $wv 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ph_new.txt || exit 1; done
timeout -k 10 120 python tools/phase_profile.py --block 0 --wave 0 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ph_new.txt || exit 1
bash tools/ab_native.sh attackfl_amd/_C_base.so 3 --steps 20 --warmup 3 > gpurun_out/ab_new2.log 2>&1; cat gpurun_out/ab_new2.log
timeout -k 10 300 python bench.py --model CNNModel --steps 20 --warmup 3 2>/dev/null | tail -1 | cut -c1-200
bash tools/ab_native.sh attackfl_amd/_C_base.so 2 --steps 20 --warmup 3 --model RNNModel > gpurun_out/ab_rnn.log 2>&1; cat gpurun_out/ab_rnn.log
