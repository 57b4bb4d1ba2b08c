#!/bin/bash
# Every mode of tools/capture_probe (HIP graph capture rules),
# one process each, into gpurun_out/capture_probe.log; the modes that may
# crash the host process run last and a crash ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/capture_probe.log
: > $L
for m in 1 2 3 4 6 7 5 9 8; do
  timeout -k 10 60 ./tools/capture_probe $m >> $L 2>&1
  rc=$?
  echo "== mode $m rc=$rc" >> $L
  [ $rc -eq 0 ] || break
done
grep -E "^mode|EndCapture|rc=|d\[0\]|status of s1 after|GraphDestroy|Synchronize\(s1\)" $L
