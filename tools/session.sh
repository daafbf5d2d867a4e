#!/bin/bash
# One parametrised GPU-box session (replaces the per-experiment r2_*/r3_*/r4_* scripts).
#   tools/session.sh TAG [step ...]
# Steps (default: tests smoke bench prof pmc):
#   tests   every -m gpu test (one pytest process; failures are recorded, the session goes on)
#   corpus  spectrum ulp corpus (tools/fft_corpus.py), in-tree build + CORPUS_VARIANTS lib_<v> builds
#   smoke   __graft_entry__.smoke()
#   bench   the default bench line (all configs, CPU legs, per-call)   -> TAG_bench.json
#   benchprof the default bench under rocprofv3 --kernel-trace --stats: the line and its trace from one
#           process -> TAG_bench.json, TAG_benchprof/, TAG_benchprof_summary.json
#   prof    per config in PROF_CFGS: rocprofv3 --kernel-trace --stats around `bench.py --config c
#           --no-sub --no-cpu --no-ulp`; the same process's JSON line is kept next to the stats, and
#           tools/prof_summary.py reduces both to TAG_prof_summary.json (timed dispatches only)
#   pmc     per config in PMC_CFGS: FETCH_SIZE and WRITE_SIZE passes (one counter per run)
#           -> tools/pmc_bytes_per_sample.py -> TAG_<c>_pmc_traffic.json
#   pct     per-call kernel trace (tools/per_call.py)
#   ab      interleaved A/B of AB_VAR over AB_VALUES (env knob, SDRGPU_TUNING=1), AB_RUNS rounds,
#           config AB_CFG                                              -> TAG_ab_<value>_<k>.json
#   ablib   interleaved A/B of the in-tree build against sdrpp_amd/lib_<v> builds (AB_LIBS; built with
#           python sdrpp_amd/build.py --variant <v> DEFINE ...)
#   sq      SQ counter sets for SQ_CFG / SQ_RX (tools/pmc_sets.sh)
#   testk   the -m gpu tests matching PYTEST_K only (a kernel change's own tests before an A/B)
#   bits    tools/bits_digest.py (output digests of the C5 / C2 chains) for the in-tree build and each
#           sdrpp_amd/lib_<v> of AB_LIBS -> TAG_bits_<v>.json (a variant must not change the bits)
#   ulpcorpus the tonal + random spectrum ulp corpus tests alone, reports kept -> TAG_reports/
# Every GPU step runs under its own timeout; the session stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
OUT=$R/gpurun_out; TAG=${1:-s}; shift; mkdir -p "$OUT"
STEPS_LIST=${*:-tests smoke bench prof pmc}
PROF_CFGS=${PROF_CFGS:-c5 c2 c3 c4 c4g}
PMC_CFGS=${PMC_CFGS:-c5 c2 c3 c4 c4g}
PSTEPS=${PSTEPS:-20}; PWARM=${PWARM:-3}
ST=$OUT/${TAG}_status.txt
st() { echo "$1 rc=$2 $(date +%T)" >> "$ST"; [ "$2" = 0 ] || exit "$2"; }
# test failures (pytest rc 1) are recorded and the session goes on; crashes / timeouts end it
st_tests() { echo "$1 rc=$2 $(date +%T)" >> "$ST"; case "$2" in 0|1) ;; *) exit "$2";; esac; }
echo "start $(date +%T) steps: $STEPS_LIST" > "$ST"
prof() {   # prof <dir> <cmd...>: rocprofv3 from /tmp (TMPDIR) with the program right after --
  local d=$1; shift
  (cd /tmp && export TMPDIR=/tmp && "$@")
}
for step in $STEPS_LIST; do
  case $step in
  tests)
    SDRGPU_REPORT_DIR=$OUT/${TAG}_reports timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 \
      --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
    st_tests tests $? ;;
  corpus)   # spectrum ulp corpus (tools/fft_corpus.py) for the in-tree build and each CORPUS_VARIANTS build
    timeout -k 10 600 python tools/fft_corpus.py > "$OUT/${TAG}_corpus.json" 2> "$OUT/${TAG}_corpus.err"
    st corpus $?
    for v in ${CORPUS_VARIANTS:-}; do
      SDRGPU_LIB_PATH=$R/sdrpp_amd/lib_$v/libsdrgpu.so timeout -k 10 600 python tools/fft_corpus.py > "$OUT/${TAG}_corpus_$v.json" 2>> "$OUT/${TAG}_corpus.err"
      st corpus_$v $?
    done ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1
    st smoke $? ;;
  bench)
    timeout -k 10 700 python bench.py ${BENCH_ARGS:-} > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
    st bench $? ;;
  benchprof)   # the default bench line and its kernel trace from ONE process (prof_summary --combined)
    prof x timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_benchprof" -o run -- \
      python3 "$R/bench.py" ${BENCH_ARGS:-} > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
    st benchprof $?
    python tools/prof_summary.py --combined "$OUT" "$TAG" > "$OUT/${TAG}_benchprof_summary.json" 2>> "$ST"
    st benchprof_summary $? ;;
  prof)
    for c in $PROF_CFGS; do
      prof x timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_$c" -o run -- \
        python3 "$R/bench.py" --config $c --no-sub --no-cpu --no-ulp --steps $PSTEPS --warmup $PWARM > "$OUT/${TAG}_prof_$c.json" 2> "$OUT/${TAG}_prof_$c.err"
      st prof_$c $?
    done
    python tools/prof_summary.py "$OUT" "$TAG" $PROF_CFGS > "$OUT/${TAG}_prof_summary.json" 2>> "$ST"
    st prof_summary $? ;;
  pmc)
    for c in $PMC_CFGS; do
      for ctr in FETCH_SIZE WRITE_SIZE; do
        prof x timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/${TAG}_pmc_${c}_$ctr" -o run -- \
          python3 "$R/bench.py" --config $c --no-sub --no-cpu --no-ulp --steps 3 --warmup 1 > "$OUT/${TAG}_pmc_${c}_$ctr.json" 2> "$OUT/${TAG}_pmc_${c}_$ctr.err"
        st pmc_${c}_$ctr $?
      done
      python tools/pmc_bytes_per_sample.py --config $c "$OUT/${TAG}_pmc_${c}_FETCH_SIZE" "$OUT/${TAG}_pmc_${c}_WRITE_SIZE" \
        "$OUT/${TAG}_${c}_pmc_traffic.json" >> "$OUT/${TAG}_pmc.log" 2>&1
      st pmc_sum_$c $?
    done ;;
  pct)
    prof x timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${TAG}_pct" -o run -- \
      python3 "$R/tools/per_call.py" 60 single > "$OUT/${TAG}_pct.log" 2>&1
    st pct $? ;;
  ab)
    for k in $(seq 1 ${AB_RUNS:-3}); do
      for v in $AB_VALUES; do
        env SDRGPU_TUNING=1 $AB_VAR=$v timeout -k 10 300 python bench.py --config ${AB_CFG:-c5} --no-sub --no-cpu --no-ulp \
          --steps ${AB_STEPS:-20} --warmup 3 > "$OUT/${TAG}_ab_${v}_$k.json" 2> "$OUT/${TAG}_ab_${v}_$k.err"
        st ab_${v}_$k $?
      done
    done
    python tools/ab_summary.py "$OUT" "$TAG" > "$OUT/${TAG}_ab_summary.txt" 2>&1 ;;
  ablib)    # interleaved A/B of library builds: the in-tree one vs sdrpp_amd/lib_<v> for v in AB_LIBS
    for k in $(seq 1 ${AB_RUNS:-3}); do
      for v in tree $AB_LIBS; do
        L=$R/sdrpp_amd/lib/libsdrgpu.so; [ "$v" = tree ] || L=$R/sdrpp_amd/lib_$v/libsdrgpu.so
        SDRGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config ${AB_CFG:-c5} --no-sub --no-cpu --no-ulp \
          --steps ${AB_STEPS:-20} --warmup 3 > "$OUT/${TAG}_ab_${v}_$k.json" 2> "$OUT/${TAG}_ab_${v}_$k.err"
        st ablib_${v}_$k $?
      done
    done
    python tools/ab_summary.py "$OUT" "$TAG" > "$OUT/${TAG}_ab_summary.txt" 2>&1 ;;
  sq)
    bash tools/pmc_sets.sh "${TAG}_sq" "${SQ_RX:-fir_mfma_kernel}" "$R/bench.py" --config ${SQ_CFG:-c3} --no-sub --no-cpu --no-ulp --steps 3 --warmup 1 >> "$OUT/${TAG}_sq.log" 2>&1
    st sq $? ;;
  testk)
    SDRGPU_REPORT_DIR=$OUT/${TAG}_reports timeout -k 10 600 python -u -m pytest tests -m gpu -k "$PYTEST_K" -v -p no:cacheprovider \
      --timeout 200 --timeout-method thread > "$OUT/${TAG}_testk.log" 2>&1
    st_tests testk $? ;;
  bits)
    for v in tree ${AB_LIBS:-}; do
      L=$R/sdrpp_amd/lib/libsdrgpu.so; [ "$v" = tree ] || L=$R/sdrpp_amd/lib_$v/libsdrgpu.so
      SDRGPU_LIB_PATH=$L timeout -k 10 300 python tools/bits_digest.py > "$OUT/${TAG}_bits_$v.json" 2> "$OUT/${TAG}_bits_$v.err"
      st bits_$v $?
    done ;;
  ulpcorpus)
    SDRGPU_REPORT_DIR=$OUT/${TAG}_reports timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu \
      -k "ulp_corpus or tonal_corpus or ulp_distribution" -v -p no:cacheprovider --timeout 400 --timeout-method thread \
      > "$OUT/${TAG}_ulpcorpus.log" 2>&1
    st_tests ulpcorpus $? ;;
  *) echo "unknown step $step" >> "$ST"; exit 2 ;;
  esac
done
echo "all done $(date +%T)" >> "$ST"
