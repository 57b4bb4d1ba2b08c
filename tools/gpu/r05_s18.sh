#!/bin/bash
# r05 session 18: the staged paper densify branch-free (all K x K slots,
# empty ones masked to +0), with (libdis_hip) and without (_nosort) the
# class-sorted order on the staged path: paper tests, A/B against HEAD.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s18_tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "paper or structured" --timeout 300 --timeout-method thread
TAILN=8 run s18_ab_paper 300 python3 tools/ab.py $D/libdis_hip_base.so:paper=1 $D/libdis_hip.so:paper=1 $D/libdis_hip_nosort.so:paper=1 $D/libdis_hip.so --rounds 8 --steps 10
cd /tmp && export TMPDIR=/tmp
run s18_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05_s18_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip.so:streams=1,paper=1 --rounds 1 --steps 3
cd $R
python3 tools/pmc_summary.py gpurun_out/r05_s18_sq/run_counter_collection.csv --match k_output --top 2
echo done
