set -o pipefail
bash tools/gpu_job.sh suite
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
rm -f gpurun_out/ph_all.txt
for b in 1 2; do for wv in 0 4; do timeout -k 10 120 python tools/phase_profile.py --block $b --wave $wv 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ph_all.txt || exit 1; done; done
for wv in 0 4; do timeout -k 10 120 python tools/phase_profile.py --block 0 --wave $wv 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ph_all.txt || exit 1; done
exit $rc
