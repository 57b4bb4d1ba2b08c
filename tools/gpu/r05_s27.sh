#!/bin/bash
# r05 session 27: auto layout, small 2-lanes-per-patch launches (<= 65,536
# patches: level 3 of a 16-pair sub-batch) with the in-kernel fallback
# kernel instead of tile-only + k_search8_fb: headline A/B, trace.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
TAILN=4 run s27_ab 400 python3 tools/ab.py $D/libdis_hip_base.so $D/libdis_hip.so --rounds 10 --steps 20
cd /tmp && export TMPDIR=/tmp
run s27_tr 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s27 -o run -- python3 $R/tools/ab.py $D/libdis_hip.so --rounds 2 --steps 5
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s27/run_kernel_trace.csv /tmp/g.csv | head -14
echo done
