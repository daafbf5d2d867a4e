# r7e: the C5 VFO tail's workgroup sizing (TAIL_PF loads per thread, last-stage outputs per workgroup)
set -o pipefail
R=$PWD; OUT=$R/gpurun_out; mkdir -p $OUT
run() {   # run TAG LIB BIGOUT k
  L=$R/sdrpp_amd/lib/libsdrgpu.so; [ "$2" = tree ] || L=$R/sdrpp_amd/lib_$2/libsdrgpu.so
  SDRGPU_LIB_PATH=$L SDRGPU_TUNING=1 SDRGPU_TAIL_BIGOUT=$3 timeout -k 10 300 python bench.py --config c5 --no-sub --no-cpu --no-ulp \
    --steps 20 --warmup 3 > $OUT/r7e_ab_$1_$4.json 2> $OUT/r7e_ab_$1_$4.err
}
for k in 1 2; do
  run tree512 tree 512 $k || exit $?
  run pf32_512 pf32 512 $k || exit $?
  run pf32_256 pf32 256 $k || exit $?
  run pf64_1024 pf64 1024 $k || exit $?
  run pf64_512 pf64 512 $k || exit $?
done
python tools/ab_summary.py $OUT r7e > $OUT/r7e_ab_summary.txt 2>&1
cd /tmp && export TMPDIR=/tmp
for v in tree pf32 pf64; do
  L=$R/sdrpp_amd/lib/libsdrgpu.so; [ "$v" = tree ] || L=$R/sdrpp_amd/lib_$v/libsdrgpu.so
  B=512; [ "$v" = pf64 ] && B=1024
  SDRGPU_LIB_PATH=$L SDRGPU_TUNING=1 SDRGPU_TAIL_BIGOUT=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r7e_prof_$v -o run -- python3 $R/bench.py --config c5 --no-sub --no-cpu --no-ulp --steps 10 --warmup 2 > $OUT/r7e_prof_$v.json 2> $OUT/r7e_prof_$v.err || exit $?
done
