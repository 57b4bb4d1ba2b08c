#!/bin/bash
# r03 session: pyramid parity with the one-sided sqrt, then the pyramid
# wave-order / rows-per-wave options re-measured on the lighter kernel.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 60 tools/sqrt_dir || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "sqrt or stage or end_to_end or interior or medium_1080p or 4k or golden" > gpurun_out/pyr_tests.log 2>&1
rc=$?; tail -5 gpurun_out/pyr_tests.log; [ $rc -eq 0 ] || exit $rc
D=optical-flow-using-dense-inverse-search_amd/disflow
SPAWN=3 bash tools/gpu/ab_pyr.sh $D/libdis_hip.so $D/libdis_hip_xcd1.so $D/libdis_hip_xcd2.so $D/libdis_hip_rows2.so
for k in 1 2 3 4; do python3 tools/trace_stats.py gpurun_out/lv$k/run_kernel_trace.csv /tmp/s$k.csv | grep -E 'pyr'; done
