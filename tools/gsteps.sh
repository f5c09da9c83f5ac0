#!/bin/bash
# GPU step runner for gpurun calls: reads "name|seconds|command" lines from the file $1 and runs each
# under its own time limit (timeout -k 10), output in $GSTEPS_OUT/<name>.log (default gpurun_out/steps).
# An ordinary failure (a test that fails: exit 1 or 2) goes on to the next step; a crash-like end
# (a time limit, an abort, a signal: exit >= 124) stops the call there, so nothing else touches the GPU.
out=${GSTEPS_OUT:-gpurun_out/steps}
mkdir -p "$out"
while IFS= read -r line || [ -n "$line" ]; do
  case "$line" in ''|'#'*) continue ;; esac
  name=${line%%|*}; rest=${line#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "[gsteps] $(date +%T) $name (limit ${to}s)"
  timeout -k 10 "$to" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc" >> "$out/rc.txt"
  echo "[gsteps] $(date +%T) $name rc=$rc"
  if [ "$rc" -ge 124 ]; then echo "[gsteps] stopping after $name (rc $rc)"; exit "$rc"; fi
done < "$1"
