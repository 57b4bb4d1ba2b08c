#!/bin/bash
# r05 session 33: paper-mode F == 0 staging box back at 80 x 80 (stride 80;
# the r05 fixed-stride change had left the 67-row box unstaged): GPU suite,
# F == 0 paper A/B and output-kernel trace against the pre-session-30 tree.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s33_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
F0="--preset slow --batch 8"
TAILN=8 run s33_ab_f0 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1,vr=0,iters=12 $D/libdis_hip.so:paper=1,vr=0,iters=12 $F0 --rounds 6 --steps 5
cd /tmp && export TMPDIR=/tmp
run s33_tr_base 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s33_base -o run -- python3 $R/tools/ab.py $D/libdis_hip_base.so:paper=1,vr=0,iters=12,streams=1 $F0 --rounds 2 --steps 3
run s33_tr_new 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s33_new -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:paper=1,vr=0,iters=12,streams=1 $F0 --rounds 2 --steps 3
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s33_base/run_kernel_trace.csv /tmp/g.csv | grep k_output
python3 tools/trace_stats.py gpurun_out/r05_s33_new/run_kernel_trace.csv /tmp/g.csv | grep k_output
echo done
