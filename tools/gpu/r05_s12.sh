#!/bin/bash
# r05 session 12: v_med3 clamp of the bilinear sample position (paper output,
# paper init, weighted densify): paper + scene tests, A/B against the staged
# build (_stg) and HEAD (_base).
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s12_tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "paper or structured" --timeout 300 --timeout-method thread
TAILN=8 run s12_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip_stg.so:paper=1 $D/libdis_hip.so:paper=1 $D/libdis_hip.so --rounds 8 --steps 10
echo done
