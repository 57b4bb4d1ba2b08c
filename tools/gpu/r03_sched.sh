#!/bin/bash
# r03 session: LLVM AMDGPU scheduler strategies for the whole library
# (parity of the finest-level cases, step A/B, per-kernel one-stream times).
# Variants: tools/build_variants.sh milp:"-mllvm -amdgpu-sched-strategy=max-ilp" \
#   iilp:"-mllvm -amdgpu-sched-strategy=iterative-ilp" mmc:"-mllvm -amdgpu-sched-strategy=max-memory-clause"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
D=optical-flow-using-dense-inverse-search_amd/disflow
for v in milp iilp mmc; do
  DISFLOW_LIB=$PWD/$D/libdis_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "medium_1080p or golden" > gpurun_out/sched_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
SPAWN=4 bash tools/gpu/ab_pyr.sh $D/libdis_hip.so $D/libdis_hip_milp.so $D/libdis_hip_iilp.so $D/libdis_hip_mmc.so > /dev/null
grep -v amdgpu.ids gpurun_out/ab.log | tail -4
for k in 1 2 3 4; do python3 tools/trace_stats.py gpurun_out/lv$k/run_kernel_trace.csv /tmp/s$k.csv | grep -E '3768320|k_pyr12|k_output'; done
