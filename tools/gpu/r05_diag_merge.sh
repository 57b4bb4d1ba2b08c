#!/bin/bash
# r05: the merged finest-level launch crashed the first 2-sub-batch call
# (host SIGSEGV). merge2 (join into the caller's stream, search, fork again)
# first, then the sub-to-sub event version: eager before graph capture.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-4}; [ $rc -eq 0 ] || exit $rc; }
SMALL="--batch 2 --width 640 --height 480 --rounds 1 --steps 1"
run dm_m2_eager 120 python3 tools/ab.py $D/libdis_hip_merge2.so:graphs=0 $SMALL
run dm_m2_graph 120 python3 tools/ab.py $D/libdis_hip_merge2.so:graphs=1 $SMALL
run dm_m2_head 150 python3 tools/ab.py $D/libdis_hip_nomerge.so $D/libdis_hip_merge2.so --rounds 6 --steps 20
run dm_m1_eager 120 python3 tools/ab.py $D/libdis_hip.so:graphs=0 $SMALL
run dm_m1_graph 120 python3 tools/ab.py $D/libdis_hip.so:graphs=1 $SMALL
echo done
