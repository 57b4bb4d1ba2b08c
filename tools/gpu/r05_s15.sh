#!/bin/bash
# r05 session 15 (final tree): GPU suite, every BASELINE config
# (tools/bench_configs.py), the headline profile round (profile_round.sh,
# TAG=r05f), and config 5's trace + counters.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-4}; [ $rc -eq 0 ] || exit $rc; }
run s15_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=12 run s15_configs 400 python3 tools/bench_configs.py --steps 10
TAG=r05f timeout -k 10 900 bash tools/gpu/profile_round.sh || exit 1
CFG5="--preset slow --width 3840 --height 2160 --batch 2"
cd /tmp && export TMPDIR=/tmp
run s15_c5tr 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05f_cfg5 -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 3
run s15_c5sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/r05f_cfg5_sq -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
run s15_c5fe 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r05f_cfg5_fetch -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
run s15_c5wr 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r05f_cfg5_write -o run -- python3 $R/tools/ab.py $D/libdis_hip.so $CFG5 --rounds 1 --steps 2
cd $R
python3 tools/pmc_summary.py gpurun_out/r05f_cfg5_sq/run_counter_collection.csv --fetch gpurun_out/r05f_cfg5_fetch/run_counter_collection.csv --write gpurun_out/r05f_cfg5_write/run_counter_collection.csv --top 12 > gpurun_out/r05f_cfg5_summary.txt
echo done
