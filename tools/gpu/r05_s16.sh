#!/bin/bash
# r05 session 16: the paper vote weight by recip_core (v_rcp_f32 + one Newton
# step, exact on [1, 2^30) per tools/color_core_check): core check, paper
# tests, A/B against HEAD.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-10}; [ $rc -eq 0 ] || exit $rc; }
run s16_core 60 ./tools/color_core_check
run s16_tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "paper or structured or colour_fast" --timeout 300 --timeout-method thread
run s16_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 $D/libdis_hip.so --rounds 8 --steps 10
echo done
