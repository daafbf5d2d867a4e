cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
SDRGPU_REPORT_DIR=gpurun_out/r2b_rep timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2b_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r2b_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
SDRGPU_LIB_PATH=$PWD/sdrpp_amd/lib_inject/libsdrgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize.py -k "c3 or ddc" -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2b_inject.log 2>&1
echo "inject rc=$?" >> gpurun_out/r2b_inject.log
exit 0
