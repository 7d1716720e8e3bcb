# Run one gpurun call, waiting out "no GPU slot free" (exit 3: nothing ran, nothing charged) up to 12
# times; any other outcome (including a failed command) is final.  gpucall.sh LOG TIMEOUT 'COMMAND'
LOG=$1; TO=$2; shift 2
for i in $(seq 12); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 150
done
echo "rc=$rc" >> $LOG
exit $rc
