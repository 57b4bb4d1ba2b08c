#!/bin/bash
# r05 session 7: is the buffer-load fallback build faster in the default
# mode (s6: 1.647 vs 1.549 ms)? Interleaved in-process and per-process A/Bs,
# one-stream kernel traces of both; lane-layout thresholds b / c.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s7_ab 300 python3 tools/ab.py $D/libdis_hip.so $D/libdis_hip_fb.so $D/libdis_hip_lvb.so $D/libdis_hip_lvc.so --rounds 8 --steps 10
run s7_spawn 500 python3 tools/ab.py --spawn 3 --rounds 3 --steps 10 $D/libdis_hip.so $D/libdis_hip_fb.so
cd /tmp && export TMPDIR=/tmp
run s7_tr_a 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s7_a -o run -- python3 $R/tools/ab.py $D/libdis_hip.so --rounds 2 --steps 5
run s7_tr_b 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s7_b -o run -- python3 $R/tools/ab.py $D/libdis_hip_fb.so --rounds 2 --steps 5
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s7_a/run_kernel_trace.csv gpurun_out/r05_s7_a/grid_stats.csv | head -16
python3 tools/trace_stats.py gpurun_out/r05_s7_b/run_kernel_trace.csv gpurun_out/r05_s7_b/grid_stats.csv | head -16
echo done
