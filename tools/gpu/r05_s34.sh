#!/bin/bash
# r05 session 34: configuration table (tools/bench_configs.py) and the default
# bench line on the tree with the session 30-33 paper-mode changes.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
TAILN=14 run s34_configs 500 python3 tools/bench_configs.py --steps 10
run s34_bench 300 python3 bench.py
echo done
