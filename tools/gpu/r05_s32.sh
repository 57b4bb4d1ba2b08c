#!/bin/bash
# r05 session 32: paper mode, both session-31 changes together (48 x 50 I1
# staging box in the output kernel, init votes loaded up front in the
# search prologue).
# GPU suite on libdis_hip, paper A/B against HEAD (_base).
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s32_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=8 run s32_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 --rounds 8 --steps 10
TAILN=8 run s32_ab_head 300 python3 tools/ab.py $D/libdis_hip_base.so $D/libdis_hip.so --rounds 6 --steps 10
cd /tmp && export TMPDIR=/tmp
run s32_tr_paper 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s32_paper -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 2 --steps 5
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s32_paper/run_kernel_trace.csv /tmp/g.csv | head -8
echo done
