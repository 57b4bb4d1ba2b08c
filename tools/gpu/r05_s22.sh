#!/bin/bash
# r05 session 22 (final tree): paper vote slots at constant offsets from the
# pixel's first covering patch, 24-bit class index multiply; full GPU suite,
# smoke, paper A/B against the previous build, the default bench line.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s22_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run s22_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
TAILN=8 run s22_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 $D/libdis_hip.so --rounds 8 --steps 10
TAILN=1 run s22_bench 400 python3 bench.py
echo done
