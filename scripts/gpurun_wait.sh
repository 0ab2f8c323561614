# Submit one gpurun call, re-submitting ONLY while the pool has no box for it
# (gpurun exit 3 / "backing off": nothing ran, nothing charged).  A call that
# ran -- whatever its result -- is never repeated.
# usage: bash scripts/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; shift 2
for i in $(seq 1 ${TRIES:-20}); do
  timeout $((lim + 600)) /usr/local/graft/bin/gpurun --timeout $lim -- "$@" > $out 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "backing off\|no free box" $out; then
    echo "[gpurun_wait] try $i: no box (rc=$rc), waiting" >> $out.wait
    sleep ${WAIT_S:-150}
    continue
  fi
  echo "[gpurun_wait] done rc=$rc after $i tries" >> $out.wait
  exit $rc
done
exit 3
