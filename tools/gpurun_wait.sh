# Submit one gpurun command, resubmitting ONLY while the pool reports that nothing ran (exit 3: no free box, or an
# infrastructure-side "transient" verdict with no run time charged); any run that reached the box is final.
#   bash tools/gpurun_wait.sh <out file> <timeout s> '<command>'
OUT=$1
TO=$2
CMD=$3
for i in $(seq 1 12); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$OUT"; then
    sleep 150
    continue
  fi
  exit $rc
done
exit $rc
