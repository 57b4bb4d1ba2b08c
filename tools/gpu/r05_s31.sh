#!/bin/bash
# r05 session 31: paper mode -- (_s48) the output kernel with a 48 x 50 I1
# staging box (LDS 26.0 -> 23.0 KB: 7 workgroups per CU instead of 6);
# (libdis_hip) the search prologue's init votes with all taps loaded up front.
# GPU suite on libdis_hip, paper A/B against HEAD (_base).
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s31_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=8 run s31_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip_s48.so:paper=1 $D/libdis_hip.so:paper=1 --rounds 8 --steps 10
cd /tmp && export TMPDIR=/tmp
run s31_tr_paper 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s31_paper -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 2 --steps 5
run s31_tr_s48 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s31_s48 -o run -- python3 $R/tools/ab.py $D/libdis_hip_s48.so:streams=1,paper=1 --rounds 2 --steps 5
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s31_paper/run_kernel_trace.csv /tmp/g.csv | head -8
python3 tools/trace_stats.py gpurun_out/r05_s31_s48/run_kernel_trace.csv /tmp/g.csv | grep k_output
echo done
