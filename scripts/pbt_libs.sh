# Per-block aggregate throughput (scripts/perblock_threads.cpp) once per
# library build in LIBS ("tree" or ablib/x.so), each linked into its own
# directory as libturbopfor_amd.so.  -> gpurun_out/${TAG}_pbt_<lib>.jsonl
# usage (on the box): LIBS="tree ablib/x.so" K=4000 THREADS="1 8 16 32" TAG=t bash scripts/pbt_libs.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for lib in ${LIBS:-tree}; do
  n=$(basename $lib .so)
  d=$R/gpurun_out/pbt_$n
  mkdir -p $d
  if [ $lib = tree ]; then cp turbopfor-cpp_amd/lib/libturbopfor_amd.so $d/; else cp $lib $d/libturbopfor_amd.so; fi
  g++ -std=c++20 -O2 -Iinclude scripts/perblock_threads.cpp -L$d -lturbopfor_amd -Wl,-rpath,$d -lpthread -o $d/pbt || exit 1
  timeout -k 10 ${PBT_TIMEOUT:-240} $d/pbt ${K:-4000} ${THREADS:-1 8 16 32} > $R/gpurun_out/${TAG:-pbt}_pbt_$n.jsonl 2>&1 || { echo "pbt $n rc=$?"; tail -3 $R/gpurun_out/${TAG:-pbt}_pbt_$n.jsonl; exit 1; }
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], 'n', d['n'], 'T', d['threads'], 'dec', d['dec_calls_per_s'], 'enc', d['enc_calls_per_s'], 'us', d['dec_us_per_call'], d['enc_us_per_call'])
" $R/gpurun_out/${TAG:-pbt}_pbt_$n.jsonl $n
done
