mkdir -p gpurun_out
for v in 1 2 4 7; do
SDRGPU_TUNING=1 SDRGPU_FFT_1M=3 SDRGPU_FFT_1M_V=$v timeout -k 10 200 python tools/c2_debug.py 32 > gpurun_out/c2dbg_v$v.log 2>&1 || exit 1
done
