#!/bin/bash
# One GPU session from named steps (replaces the r03 one-off session scripts):
#   tools/gpu/session.sh <step> [<step> ...]
# Steps (each under its own time limit; a crash, abort or timeout ends the
# session, a plain test / A/B failure too):
#   tests[=<pytest -k expr>]     GPU suite (or a subset), one process
#   ab=<lib[:opts]>,<lib>,...    interleaved whole-step A/B (tools/ab.py, one process)
#   abspawn=<lib>,<lib>,...      the same, one process per variant and round (4 rounds)
#   levels=<lib>,<lib>,...       per-kernel one-stream durations (rocprof kernel trace)
#   pmc=<lib>                    SQ counters of the top kernels (tools/gpu/pmc_sq.sh; CTRS= to override)
#   bench                        bench.py default line
#   smoke                        __graft_entry__.smoke()
#   tool=<name> [args]           a built tools/ binary (e.g. tool=issue_mix)
#   py=<script> [args]           a python script of the repo (e.g. py="tools/bench_configs.py --configs colour")
# Libraries are paths relative to the package's disflow/ (e.g. libdis_hip_x.so);
# build variants first on the CPU: tools/build_variants.sh name:"-DFLAG=1".
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
D=optical-flow-using-dense-inverse-search_amd/disflow
libs() { local out=(); IFS=, read -ra a <<< "$1"; for v in "${a[@]}"; do out+=("$D/$v"); done; echo "${out[@]}"; }
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-12}
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
n=0
for s in "$@"; do
  n=$((n+1)); k=${s%%=*}; v=${s#*=}
  case $k in
    tests) if [ "$s" = tests ]; then run s${n}_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
           else run s${n}_tests 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "$v"; fi ;;
    ab) run s${n}_ab 600 python3 tools/ab.py $(libs "$v") --rounds 8 --steps 10 ;;
    abspawn) run s${n}_abspawn 900 python3 tools/ab.py --spawn 4 --rounds 3 --steps 10 $(libs "$v") ;;
    levels) run s${n}_levels 600 bash tools/gpu/levels.sh $(libs "$v") ;;
    pmc) run s${n}_pmc 300 bash tools/gpu/pmc_sq.sh $(libs "$v") ;;
    bench) run s${n}_bench 400 python bench.py ;;
    smoke) run s${n}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tool) run s${n}_$(echo "$v" | cut -d' ' -f1) 300 ./tools/$v ;;
    py) run s${n}_$(basename "$(echo "$v" | cut -d' ' -f1)" .py) 600 python3 $v ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
