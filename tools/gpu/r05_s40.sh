#!/bin/bash
# r05 session 40: 64 x 32 output tiles at F == 0 -- paper mode only (_p0) or
# both modes (libdis_hip, _all0): GPU suite on libdis_hip, F == 0 A/B in both
# modes and the F = 1 paper step against HEAD (_base).
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s40_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
F0="--preset slow --batch 8 --rounds 6 --steps 5"
TAILN=8 run s40_ab_f0_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1,vr=0,iters=12 $D/libdis_hip_p0.so:paper=1,vr=0,iters=12 $D/libdis_hip_all0.so:paper=1,vr=0,iters=12 $F0
TAILN=8 run s40_ab_f0_ref 300 python3 tools/ab.py $D/libdis_hip_base.so:vr=0,iters=12 $D/libdis_hip_p0.so:vr=0,iters=12 $D/libdis_hip_all0.so:vr=0,iters=12 $F0
TAILN=8 run s40_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip_all0.so:paper=1 --rounds 6 --steps 10
echo done
