#!/bin/bash
# queue a gpurun call: retry only while the pool reports no free box / busy slots / back-off
# (nothing ran, nothing charged); any other outcome is final.  usage: gq.sh <out> <timeout> <cmd>
out=$1; to=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  if grep -q -E "no free box right now|GPU slot\(s\) on this pod are busy|is backing off|stopped responding while being prepared" "$out"; then
    w=$(grep -o -E "retry in [0-9]+s" "$out" | grep -o -E "[0-9]+" | head -1); sleep $(( ${w:-120} > 60 ? ${w:-120} : 60 ))
    continue
  fi
  break
done
