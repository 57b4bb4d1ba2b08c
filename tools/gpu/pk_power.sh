#!/bin/bash
# scalar vs packed f32 VALU at full load: time per launch, clock and power
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in scalar pk scalar pk; do
  timeout -k 10 60 ./tools/pk_power $m 16 > gpurun_out/pk_$m.log 2>&1 &
  pid=$!
  sleep 6
  for i in 1 2 3 4; do
    timeout 20 amd-smi metric -g 0 --power --clock 2>&1 | grep -E "SOCKET_POWER|^ *CLK:" | head -2 | tr -s ' ' | tr '\n' ' '; echo
    sleep 1.5
  done
  wait $pid; rc=$?; cat gpurun_out/pk_$m.log; [ $rc -eq 0 ] || exit $rc
done
