set -e
mkdir -p gpurun_out
cp attackfl_amd/_C.so /tmp/_C_prod.so
for x in 0 1 2 4 8 16; do
  cp abl/_C_$x.so attackfl_amd/_C.so
  timeout -k 10 100 python -u tools/phase_profile.py --clients 8 --block 1 > gpurun_out/abl_$x.log 2>&1
done
cp /tmp/_C_prod.so attackfl_amd/_C.so
