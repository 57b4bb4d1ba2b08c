#!/bin/bash
# r05 session 8: GPU suite, every BASELINE config (tools/bench_configs.py,
# with config 1's CPU path and config 5's refinement roofline), then the
# profile round of this tree (tools/gpu/profile_round.sh, TAG=r05).
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-4}; [ $rc -eq 0 ] || exit $rc; }
run s8_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
TAILN=12 run s8_configs 400 python3 tools/bench_configs.py --steps 10
TAG=r05 timeout -k 10 900 bash tools/gpu/profile_round.sh
