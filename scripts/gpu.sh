# One parametrised GPU-box runner (replaces the per-call gpu_r3*.sh one-offs).
# usage (on the box, via gpurun):  TAG=r4a bash scripts/gpu.sh STEP [STEP ...]
# Every step runs under its own time limit; the first failing step ends the call.
#   tests[=K]        pytest -m gpu (optionally -k K)          -> ${TAG}_tests.log
#   smoke            __graft_entry__.py smoke                  -> ${TAG}_smoke.log
#   bench:WL[:ARGS]  bench.py --workload WL (ARGS: comma list)  -> ${TAG}_bench_WL.json
#   prof:WL          rocprofv3 --kernel-trace --stats of a bench -> ${TAG}_WL_prof/
#   pmc:WL           FETCH_SIZE and WRITE_SIZE passes (separate runs) + pmc_traffic.py
#                    -> gpurun_out/pmc_traffic.json (starts from profiles/pmc_traffic.json)
#   ab:WL            LIBS="tree ablib/x.so" ENVS="A=1 A=2" ROUNDS=2: bench per library build x env
#   libs:SCRIPT[:ARGS] python SCRIPT once per library build in LIBS     -> ${TAG}_SCRIPT.log
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (comma list)           -> ${TAG}_SCRIPT.log
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
T=${TAG:-r4}
O=$R/gpurun_out
fail() { echo "$1 rc=$2"; [ -f "$3" ] && tail -${4:-25} "$3"; exit 1; }
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  case $kind in
    tests|tests=*)
      k=${step#tests}; k=${k#=}
      timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${k:+-k "$k"} > $O/${T}_tests.log 2>&1 || fail tests $? $O/${T}_tests.log 40
      tail -1 $O/${T}_tests.log ;;
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > $O/${T}_smoke.log 2>&1 || fail smoke $? $O/${T}_smoke.log
      tail -1 $O/${T}_smoke.log ;;
    bench)
      wl=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --workload $wl ${a//,/ } > $O/${T}_bench_$wl.json 2> $O/${T}_bench_$wl.err || fail "bench $wl" $? $O/${T}_bench_$wl.err
      tail -1 $O/${T}_bench_$wl.json ;;
    prof)
      wl=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${T}_${wl}_prof -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline ${a//,/ } > $O/${T}_${wl}_under_rocprof.json 2> $O/${T}_${wl}_prof.err) || fail "prof $wl" $? $O/${T}_${wl}_prof.err
      tail -1 $O/${T}_${wl}_under_rocprof.json
      python3 -c "
import csv,glob,sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
" $O/${T}_${wl}_prof ;;
    pmc)
      wl=$rest
      [ -f $O/pmc_traffic.json ] || cp profiles/pmc_traffic.json $O/pmc_traffic.json
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $c -d $O/pmc_${wl}_$c -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_pmc_${wl}_$c.json 2>&1) || fail "pmc $wl $c" $? $O/bench_pmc_${wl}_$c.json
      done
      python3 scripts/pmc_traffic.py $wl $O/pmc_${wl}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${wl}_WRITE_SIZE/run_counter_collection.csv 10000000 $O/pmc_traffic.json ${LABEL:-$T} || fail "pmc_traffic $wl" $?
      if [ $wl = c4 ]; then
        python3 scripts/pmc_traffic.py c4_64 $O/pmc_${wl}_FETCH_SIZE/run_counter_collection.csv $O/pmc_${wl}_WRITE_SIZE/run_counter_collection.csv 10000000 $O/pmc_traffic.json ${LABEL:-$T} || fail "pmc_traffic c4_64" $?
      fi ;;
    ab)
      wl=$rest
      for i in $(seq ${ROUNDS:-2}); do
        for lib in ${LIBS:-tree}; do
         for ev in ${ENVS:-none}; do
          if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
          n=$(basename $lib .so); [ $ev = none ] || n=${n}_${ev//=/}
          timeout -k 10 240 env ${ev/#none/TPF_AB=0} python bench.py --workload $wl --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-probes ${BARGS} > $O/${T}_ab_${wl}_${n}_$i.json 2> $O/${T}_ab_${wl}_${n}_$i.err || fail "ab $n" $? $O/${T}_ab_${wl}_${n}_$i.err 5
          python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; r=d['roofline']; print(sys.argv[3], sys.argv[2], d['value'], 'ms', r.get('kernel_ms_avg'), 'verified', c.get('verified'), {k: v for k, v in c.items() if k.endswith('per_s')})" $O/${T}_ab_${wl}_${n}_$i.json $n $wl
         done
        done
      done ;;
    libs)
      # python SCRIPT ARGS once per library build in LIBS (TPF_LIB), ROUNDS times
      s=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      for i in $(seq ${ROUNDS:-2}); do
        for lib in ${LIBS:-tree}; do
          if [ $lib = tree ]; then unset TPF_LIB; else export TPF_LIB=$R/$lib; fi
          timeout -k 10 ${PY_TIMEOUT:-300} python -u $s ${a//,/ } >> $O/${T}_$(basename $s .py).log 2>&1 || fail "libs $s $lib" $? $O/${T}_$(basename $s .py).log
          tail -1 $O/${T}_$(basename $s .py).log
        done
      done
      unset TPF_LIB ;;
    py)
      s=${rest%%:*}; a=${rest#*:}; [ "$a" = "$rest" ] && a=""
      timeout -k 10 ${PY_TIMEOUT:-300} python -u $s ${a//,/ } > $O/${T}_$(basename $s .py).log 2>&1 || fail "py $s" $? $O/${T}_$(basename $s .py).log
      tail -${PY_TAIL:-15} $O/${T}_$(basename $s .py).log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
