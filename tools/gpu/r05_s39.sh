#!/bin/bash
# r05 session 39: paper-mode output tiles of 64 x 32 (LDS 23.0 -> 14.3 KB at
# F >= 1: 8 workgroups per CU; F == 0 69.6 -> 39.4 KB): GPU suite,
# paper A/B (F = 1 and F = 0) against HEAD, output-kernel trace and counters.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s39_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=8 run s39_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 --rounds 8 --steps 10
TAILN=8 run s39_ab_f0 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1,vr=0,iters=12 $D/libdis_hip.so:paper=1,vr=0,iters=12 --preset slow --batch 8 --rounds 6 --steps 5
cd /tmp && export TMPDIR=/tmp
run s39_tr_paper 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05_s39_paper -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 2 --steps 5
run s39_sq_paper 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s39_sqp -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 1 --steps 3
cd $R
python3 tools/trace_stats.py gpurun_out/r05_s39_paper/run_kernel_trace.csv /tmp/g.csv | grep k_output
python3 tools/pmc_summary.py gpurun_out/r05_s39_sqp/run_counter_collection.csv --match k_output --top 1
echo done
