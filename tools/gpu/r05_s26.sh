#!/bin/bash
# r05 session 26: the final HEAD build -- full GPU suite and smoke.
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids $R/gpurun_out/$name.log | tail -${TAILN:-4}; [ $rc -eq 0 ] || exit $rc; }
run s26_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run s26_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
echo done
