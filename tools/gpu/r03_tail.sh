#!/bin/bash
# r03 session: register/DPP pyramid tail (k_pyr_tail_reg) -- GPU parity, then
# A/B against the LDS tail and per-kernel durations (one stream). Variants:
#   tools/build_variants.sh tailold:"-DDIS_TAIL_REG=0" tail4:"-DDIS_TAIL_REG_TPW=4" \
#     wg2:"-DDIS_PYR12_WG=2" wg4:"-DDIS_PYR12_WG=4" wg8:"-DDIS_PYR12_WG=8"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -5 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit $rc
D=optical-flow-using-dense-inverse-search_amd/disflow
SPAWN=3 bash tools/gpu/ab_pyr.sh $D/libdis_hip.so $D/libdis_hip_tailold.so $D/libdis_hip_tail4.so $D/libdis_hip_wg2.so $D/libdis_hip_wg4.so $D/libdis_hip_wg8.so > /dev/null
grep -v amdgpu.ids gpurun_out/ab.log | tail -4
for k in 1 2 3 4 5 6; do echo "== $k"; python3 tools/trace_stats.py gpurun_out/lv$k/run_kernel_trace.csv /tmp/s$k.csv | grep -E 'pyr'; done
