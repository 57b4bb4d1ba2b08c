#!/bin/bash
# r05 session 37: final-tree check -- GPU suite, smoke(), default bench line,
# kernel-trace statistics of the bench command.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-6}; [ $rc -eq 0 ] || exit $rc; }
run s37_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run s37_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run s37_bench 300 python3 bench.py
cd /tmp && export TMPDIR=/tmp
run s37_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_s37_prof -o run -- python3 $R/bench.py --steps 20 --warmup 5
cd $R
echo done
