# A/B the decode kernel variants on one box (TPF_DEC_VARIANT), then the tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for v in ${VARIANTS:-0 1}; do
  TPF_DEC_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "variant $v rc=$?"; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('variant $v', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_avg'], d['config']['verified'])"
  grep sweep gpurun_out/ab_$v.err | awk '{print $2, $5, $6}' | tr '\n' ' '; echo
done
if [ -n "$RUN_TESTS" ]; then timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/pytest_ab.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_ab.log; fi
