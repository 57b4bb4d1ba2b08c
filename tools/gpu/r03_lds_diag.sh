#!/bin/bash
# r03 session: where the finest search's issue cycles go -- one PMC pass of
# LDS-pipe and VALU-activity counters over the profile-round bench command.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; R=$GRAFT_REPO_ROOT
BENCH="$R/bench.py --steps 10 --warmup 5 --warmup-floor 0 --no-cpu-baseline --no-tolerance-mode --no-pipelined"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r03_ldsdiag -o run -- python3 $BENCH > $R/gpurun_out/ldsdiag.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
