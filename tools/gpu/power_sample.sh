#!/bin/bash
# Clock and power of the GPU while bench.py's headline step runs (read-only
# queries): is the VALU-bound search running at the power limit?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --steps 40000 --warmup 5 --no-cpu-baseline --no-tolerance-mode --no-pipelined --no-kernel-timing > gpurun_out/power_bench.log 2>&1 &
pid=$!
sleep 30
for i in $(seq 1 10); do
  echo "--- sample $i $(date +%T)"
  timeout 20 amd-smi metric -g 0 --power --clock 2>&1 | grep -E "SOCKET_POWER|^ *CLK:" | head -3
  sleep 1
done > gpurun_out/power.log 2>&1
timeout 20 amd-smi static -g 0 --limit >> gpurun_out/power.log 2>&1
wait $pid; echo "bench rc=$?"; tail -1 gpurun_out/power_bench.log | cut -c1-160
cat gpurun_out/power.log | head -60
