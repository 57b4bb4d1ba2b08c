#!/bin/bash
# r03 session: search taps read ahead during the solve (DIS_TAP_PREFETCH) --
# parity of the variant builds, then A/B against the default and the finest
# launch's duration (one stream).
# Variants: tools/build_variants.sh pf2:"-DDIS_TAP_PREFETCH=1 -DDIS_TAP_PREFETCH_ROWS=2" \
#             pf3:"-DDIS_TAP_PREFETCH=1 -DDIS_TAP_PREFETCH_ROWS=3"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
D=optical-flow-using-dense-inverse-search_amd/disflow
for v in pf2 pf3; do
  DISFLOW_LIB=$PWD/$D/libdis_hip_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "end_to_end or medium_1080p or 4k or golden or lanes or paper or outliers or fallback" > gpurun_out/pf_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc"; tail -2 gpurun_out/pf_$v.log; [ $rc -eq 0 ] || exit $rc
done
SPAWN=4 bash tools/gpu/ab_pyr.sh $D/libdis_hip.so $D/libdis_hip_pf2.so $D/libdis_hip_pf3.so > /dev/null
grep -v amdgpu.ids gpurun_out/ab.log | tail -3
for k in 1 2 3; do python3 tools/trace_stats.py gpurun_out/lv$k/run_kernel_trace.csv /tmp/s$k.csv | grep -E '3768320|983040'; done
